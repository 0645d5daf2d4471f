"""Occupancy guard (no GPU needed): every path-kernel instantiation in the built
code object must fit 16 waves per CU (<= 128 VGPRs, no scratch in the product
variants) -- the global-memory variant once drifted to 130 VGPRs and lost a
quarter of its occupancy."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_path_kernels_fit_16_waves_per_cu(tmp_path):
    csrc = os.path.join(ROOT, "montecarlopathtracer_amd", "csrc")
    s_file = tmp_path / "render.s"
    cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "--cuda-device-only", "-S", "-O3",
           "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fno-slp-vectorize",
           "-I" + os.path.join(ROOT, "include"), os.path.join(csrc, "render.hip"), "-o", str(s_file)]
    if not os.path.exists(cmd[0]):
        pytest.skip("hipcc not available")
    subprocess.run(cmd, check=True, capture_output=True)
    text = s_file.read_text()
    metas = re.findall(r"\.name:\s+(\S*path_kernel\S*)\n(?:.*\n){0,40}?\s+\.vgpr_count:\s+(\d+)", text)
    assert metas, "no path_kernel metadata found"
    for name, vgpr in metas:
        assert int(vgpr) <= 128, (name, vgpr)
    scratch = re.findall(r"\.amdhsa_kernel (\S*path_kernel\S*)\n(?:.*\n)*?\s+\.amdhsa_private_segment_fixed_size (\d+)",
                         text)
    for name, size in scratch:
        if "ELb0ELb" in name:        # product variants (the DBG unit-counter ones may spill)
            assert int(size) == 0, (name, size)
