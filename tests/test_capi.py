"""The C ABI boundary (include/mcpt.h) without a GPU: the library loads,
exports every declared symbol, host-only entry points behave, errors surface
as codes + messages, and the tile-sharding map is a partition of the image."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(ROOT, "include", "mcpt.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mcpt_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol(mcpt):
    lib = C.CDLL(os.path.join(ROOT, "montecarlopathtracer_amd", "lib", "libmcpt.so"))
    names = _declared()
    assert len(names) >= 25
    for n in names:
        assert hasattr(lib, n), n
    from montecarlopathtracer_amd import _capi
    assert sorted(_capi.declared_symbols()) == names      # the binding covers the whole header


def test_abi_version_and_defaults(mcpt):
    from montecarlopathtracer_amd._capi import RenderParamsC, lib
    assert lib().mcpt_abi_version() == 9
    p = RenderParamsC()
    lib().mcpt_render_params_default(C.byref(p))
    # CV/stdafx.h:41-46, CUTracer.cu:189,212,349-351
    assert (p.width, p.height, p.spp, p.max_depth) == (800, 600, 100, 7)
    assert p.illum == 10.0 and p.fov_deg == 60.0
    assert list(p.eye) == [0, 5, 17] and list(p.dir) == [0, 0, -1] and list(p.up) == [0, 1, 0]
    assert p.fresnel_kd == 1 and p.tile == 8 and p.mode == 0 and p.pipeline == 0
    q = RenderParamsC()
    lib().mcpt_render_params_quinengine(C.byref(q))
    # QE/RTX/GraphicsRTX.cpp:173-193, QE/Shader/rtx.hlsl:400
    assert (q.mode, q.spp, q.max_depth, q.fresnel_kd) == (1, 1, 5, 0)
    assert q.fov_deg == 45.0 and list(q.eye) == [0, 5, 17] and q.illum == 1.0
    assert (q.width, q.height) == (640, 480)                 # the QE window, QE/Main.cpp:11
    # scheduling fields default to 0 = automatic
    for f in ("wf_streams", "wf_refill", "wf_group_shift", "ready_thresh", "tail_units_per_lane", "tail_units",
              "wf_mem_limit", "force_peer_copy"):
        assert getattr(p, f) == 0 and getattr(q, f) == 0, f
    # the Python mirror agrees with the C defaults
    r = mcpt.RenderParams.for_quinengine().to_c()
    for f in ("mode", "spp", "max_depth", "fresnel_kd", "fov_deg", "illum", "width", "height"):
        assert getattr(r, f) == getattr(q, f), f


def test_host_scene_errors(mcpt):
    m = mcpt.ObjModel(mcpt.scene_path("scene01"))
    s = mcpt.Scene(m, host_only=True)
    with pytest.raises(mcpt.McptError) as e:
        s.render(mcpt.RenderParams(width=8, height=8, spp=1))
    assert e.value.code == -1 and "host-only" in str(e.value)
    from montecarlopathtracer_amd._capi import lib
    assert lib().mcpt_render(None, None, None, None) == -1
    assert b"NULL" in lib().mcpt_last_error()


@pytest.mark.parametrize("W,H,T,N", [(64, 48, 8, 1), (70, 50, 8, 3), (1024, 1024, 8, 8), (33, 17, 16, 4), (5, 5, 8, 7)])
def test_shards_partition_the_image(mcpt, W, H, T, N):
    seen = np.zeros((H, W), np.int32)
    total = 0
    for r in range(N):
        p = mcpt.RenderParams(width=W, height=H, tile=T, shard_count=N, shard_index=r)
        xy = p.shard_pixels()
        assert xy.shape[0] == p.output_pixels()
        ok = xy[:, 0] >= 0
        seen[xy[ok, 1], xy[ok, 0]] += 1
        total += ok.sum()
        # packed order: tile-major, row-major inside a tile
        if ok.sum():
            first = xy[ok][0]
            assert first[0] % T == 0 and first[1] % T == 0
    assert total == W * H and (seen == 1).all()


def test_pw_tracer_adapter_compiles_and_links(mcpt):
    """include/mcpt_pw_tracer.hpp: reference-style PW::Tracer calls compile and link
    against libmcpt.so (run on the GPU in tests/test_gpu_parity.py)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "cpp"))
    import build_dropin
    assert os.path.exists(build_dropin.build())
    assert os.path.exists(build_dropin.build("qe_viewer"))      # include/mcpt_qe_viewer.hpp


def test_struct_layouts_match_header(mcpt, tmp_path):
    """ctypes mirrors (_capi.py) have the sizes and field offsets of include/mcpt.h."""
    import ctypes
    import subprocess
    from montecarlopathtracer_amd import _capi
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    structs = {"mcpt_render_params": _capi.RenderParamsC, "mcpt_render_stats": _capi.RenderStats,
               "mcpt_scene_info": _capi.SceneInfo, "mcpt_model_info": _capi.ModelInfo,
               "mcpt_model_desc": _capi.ModelDesc, "mcpt_plan_info": _capi.PlanInfo,
               "mcpt_scene_options": _capi.SceneOptions}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "mcpt.h"', 'int main(void) {']
    for cname, py in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", inc, str(src), "-o", str(exe)], check=True)
    out = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                         check=True).stdout.split("\n") if l)
    for cname, py in structs.items():
        assert int(out[cname]) == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(out[f"{cname}.{f}"]) == getattr(py, f).offset, (cname, f)


def test_fastdiv_equals_integer_division():
    """The work-unit decode's multiply-high division (render_launch.hpp FastDiv)
    equals n / d: every divisor up to 70000 and 40000 random ones, dividends at
    the edges, around multiples and random."""
    import subprocess
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "cpp"))
    import build_dropin
    out = subprocess.run([build_dropin.build("fastdiv_probe")], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout + out.stderr
