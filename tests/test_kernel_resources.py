"""Occupancy guard (no GPU needed), read from the code object that ships.

The gfx950 code objects are taken out of the built libmcpt.so itself (its
.hip_fatbin section: clang offload bundles, one per HIP translation unit), so
the check covers exactly the binary the product loads -- same flags, including
_build.py's max-ILP scheduler.  Every persistent kernel must fit its launch
shape: the megakernel variants and the wavefront extend kernels run 16 waves
per CU (<= 128 VGPRs + AGPRs per lane, no scratch in the product variants);
the global-memory variant once drifted to 130 VGPRs and lost a quarter of its
occupancy.
"""
import os
import re
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _code_objects(lib, tmp_path):
    fatbin = tmp_path / "fatbin.bin"
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fatbin}", lib,
                    str(tmp_path / "stripped.so")], check=True, capture_output=True)
    blob = fatbin.read_bytes()
    out = []
    for m in re.finditer(re.escape(MAGIC), blob):
        base = m.start()
        n, p = struct.unpack_from("<Q", blob, base + 24)[0], base + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", blob, p)
            p += 24
            triple = blob[p:p + tl].decode()
            p += tl
            if "gfx950" in triple and size:
                assert blob[base + off:base + off + 4] == b"\x7fELF", "compressed or unknown bundle"
                f = tmp_path / f"co{len(out)}.elf"
                f.write_bytes(blob[base + off:base + off + size])
                out.append(f)
    return out


def _kernels(co):
    txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", str(co)], check=True,
                         capture_output=True, text=True).stdout
    ks = {}
    for block in re.split(r"\n  - (?=\.agpr_count)", txt):
        name = re.search(r"\.name:\s+(\S+)", block)
        if not name:
            continue
        get = lambda k: int(re.search(rf"\.{k}:\s+(\d+)", block).group(1))  # noqa: E731
        ks[name.group(1)] = {"vgpr": get("vgpr_count"), "agpr": get("agpr_count"),
                             "scratch": get("private_segment_fixed_size")}
    return ks


def test_shipped_kernels_fit_16_waves_per_cu(tmp_path):
    if not os.path.exists(os.path.join(LLVM, "llvm-readelf")):
        pytest.skip("ROCm llvm tools not available")
    import importlib.util
    spec = importlib.util.spec_from_file_location("_b", os.path.join(ROOT, "montecarlopathtracer_amd", "_build.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    lib = b.build()                       # no-op when libmcpt.so is up to date
    kernels = {}
    for co in _code_objects(lib, tmp_path):
        kernels.update(_kernels(co))
    path = {k: v for k, v in kernels.items() if "path_kernel" in k}
    extend = {k: v for k, v in kernels.items() if "wf_extend" in k}
    assert len(path) == 18, sorted(path)  # 3 layouts x (DBG, QE, COUNT) variants
    # 2 layouts x (lean, counting), + the wave-coherent bounce-0 extend (lean, counting)
    assert len(extend) == 6, sorted(extend)
    for name, r in {**path, **extend}.items():
        assert r["vgpr"] + r["agpr"] <= 128, (name, r)
        # product variants: the DBG unit-counter megakernels (template arg 4 true) may spill
        if "wf_extend" in name or re.search(r"path_kernelILb[01]ELi\d+ELi\d+ELb0E", name):
            assert r["scratch"] == 0, (name, r)
    # the residency the wavefront's schedule is built on: the
    # lean extend of global-memory scenes (template <LAY 0, S, 256, lean>) at
    # <= 80 VGPRs -- six workgroups per CU -- and the LDS
    # scenes' (LAY 1) at <= 88 beside two <= 80-VGPR shade waves per SIMD
    g_lean = [r for k, r in extend.items() if re.search(r"wf_extendILi0ELi\d+ELi256ELb0EE", k)]
    l_lean = [r for k, r in extend.items() if re.search(r"wf_extendILi1ELi4ELi1024ELb0EE", k)]
    assert len(g_lean) == 1 and len(l_lean) == 1, sorted(extend)
    assert g_lean[0]["vgpr"] <= 80 and l_lean[0]["vgpr"] <= 88, (g_lean, l_lean)
    # (both shades: queue order and the material sort)
    shade = [r for k, r in kernels.items() if re.search(r"wf_shade_slotsILi512E", k)]
    assert len(shade) == 4 and all(r["vgpr"] <= 80 for r in shade), shade
    # the other wavefront kernels run at most 512 VGPRs' worth of waves; keep them spill-free
    for name, r in kernels.items():
        if "wf_" in name:
            assert r["scratch"] == 0, (name, r)


def _disasm(lib, tmp_path):
    """kernel name -> its instruction lines (mnemonic first), from the shipped code objects"""
    out = {}
    for co in _code_objects(lib, tmp_path):
        txt = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", str(co)], check=True,
                             capture_output=True, text=True).stdout
        cur = None
        for line in txt.splitlines():
            m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line.strip())
            if m:
                cur = m.group(1)
                out[cur] = []
            elif cur and line.strip() and not line.strip().startswith(";"):
                out[cur].append(line.strip())
    return out


def test_codegen_flags_still_do_their_job(tmp_path):
    """each per-source LLVM option in _build.py was adopted
    for a measured gain; this pins, in the shipped code objects, the code
    property each one produces, so a toolchain change that silently drops it
    fails here.  Counts with / without the option (ROCm 7.2, measured by
    compiling the source with the option removed):
    * -amdgpu-set-wave-priority=1 (wavefront sources): an `s_setprio 3` around
      the first vector-memory loads of every extend kernel (the source itself
      only uses priorities 0 and 1): 1 / 0;
    * -unroll-threshold=2000 (wavefront.hip, render.hip): the global-memory
      variants' capped descent unrolled -- 12 fp16 box-bound conversions per
      step (two child boxes), so 12 x cap of them (caps 6 / 5: 72 and 60,
      one step's 12 without the option);
    * -two-entry-phi-node-folding-threshold=8 (wavefront.hip): if-diamonds of
      the global extend folded into selects -- exec-mask regions
      (`s_and_saveexec_b64`) in the lean queue-order global extend: 83 / 103;
    * -enable-gvn-hoist (render.hip): float products common to both sides of
      a branch hoisted -- `v_mul_f32_e32` in the lean LDS / global megakernels:
      181 / 184 and 277 / 281;
    * -structurizecfg-skip-uniform-regions=1 (wavefront_primary.hip): uniform
      branches of the bounce-0 packet walk kept as scalar branches instead of
      exec-mask regions -- `s_cbranch_vccz` in its lean kernel: 5 / 14."""
    if not os.path.exists(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("ROCm llvm tools not available")
    import importlib.util
    spec = importlib.util.spec_from_file_location("_b", os.path.join(ROOT, "montecarlopathtracer_amd", "_build.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    lib = b.build()
    k = _disasm(lib, tmp_path)

    def one(pat):
        m = [n for n in k if re.search(pat, n)]
        assert len(m) == 1, (pat, m)
        return k[m[0]]

    def count(ins, prefix):
        return sum(1 for x in ins if x.split()[0].startswith(prefix))

    extends = [n for n in k if "wf_extend" in n]
    assert extends
    for n in extends:
        assert any(x.startswith("s_setprio 3") for x in k[n]), n
    g_ext = one(r"wf_extendILi0ELi\d+ELi256ELb0EE")       # global layout, lean
    mk_glob = one(r"path_kernelILb0ELi8ELi256ELb0ELb1ELb0E")   # global layout, lean megakernel
    mk_lds = one(r"path_kernelILb1ELi4ELi1024ELb0ELb0ELb0E")   # LDS layout, lean megakernel
    assert count(g_ext, "v_cvt_f32_f16") >= 12 * 6               # MCPT_WF_DESCENT_CAP_GLOBAL
    assert count(mk_glob, "v_cvt_f32_f16") >= 12 * 5             # MCPT_DESCENT_CAP_GLOBAL
    assert count(g_ext, "s_and_saveexec_b64") <= 93
    assert count(mk_lds, "v_mul_f32_e32") <= 182 and count(mk_glob, "v_mul_f32_e32") <= 279
    prim = one(r"wf_extend_primaryILi4ELi1024ELb0E")
    assert count(prim, "s_cbranch_vccz") <= 9
