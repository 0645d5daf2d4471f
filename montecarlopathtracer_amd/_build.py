"""Build libmcpt.so (HIP for gfx950 + C++ host) in-tree with hipcc.

Output: montecarlopathtracer_amd/lib/libmcpt.so.  Every translation unit is
compiled with -ffp-contract=off and without fast-math: the kernel's float
arithmetic must round exactly as the specification.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, os.environ.get("MCPT_LIB_NAME", "libmcpt.so"))
SOURCES = ["host_model.cpp", "kd_cache.cpp", "capi.cpp", "render.hip", "wavefront.hip", "wavefront_primary.hip"]
# per-source code generation (wavefront_primary.hip: the bounce-0 packet extend's
# wave-uniform control flow as scalar branches; render.hip: GVN hoisting,
# megakernel +1.4%, no effect on the wavefront kernels, and the global-memory
# variants' capped descent unrolled (C4 megakernel +2.1%); the wavefront kernels:
# wave priority raised around their vector-memory loads, C2 +0.4%, and
# if-diamonds of up to 8 instructions folded into selects and the capped
# descent unrolled -- only the global-memory extends change, C4 +0.9% and +3.0%)
_WF_FLAGS = ["-mllvm", "-amdgpu-set-wave-priority=1", "-mllvm", "-two-entry-phi-node-folding-threshold=8",
             "-mllvm", "-unroll-threshold=2000"]
SOURCE_FLAGS = {"wavefront_primary.hip": ["-mllvm", "-structurizecfg-skip-uniform-regions=1"] + _WF_FLAGS,
                "wavefront.hip": _WF_FLAGS,
                "render.hip": ["-mllvm", "-enable-gvn-hoist", "-mllvm", "-unroll-threshold=2000"]}
HEADERS = ["host_model.hpp", "mcpt_device.hpp", "render_launch.hpp", "trace_device.hpp", "half_box.hpp"]
ARCH = os.environ.get("MCPT_OFFLOAD_ARCH", "gfx950")

COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-fno-slp-vectorize", "-Wall",
          "-I" + os.path.join(ROOT, "include")] + os.environ.get("MCPT_EXTRA_FLAGS", "").split()


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "mcpt.h"),
                                                                 os.path.abspath(__file__)]   # flags
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    os.makedirs(os.path.join(LIBDIR, "obj"), exist_ok=True)
    hipcc = _hipcc()

    def compile_one(src):
        obj = os.path.join(LIBDIR, "obj", os.path.basename(LIB) + "." + src + ".o")
        # max-ILP machine scheduling for the kernels: +1.2% C2, +1.5% C4, +0.9% wavefront
        # (the default occupancy-driven scheduler gains nothing: occupancy is fixed by LDS)
        sched = os.environ.get("MCPT_SCHED", "max-ilp")   # A/B builds only
        lang = (["-x", "hip", f"--offload-arch={ARCH}", "-mllvm", f"-amdgpu-sched-strategy={sched}"]
                if src.endswith(".hip")
                else ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"])
        cmd = [hipcc] + lang + COMMON + SOURCE_FLAGS.get(src, []) + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
        return obj

    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = LIB + f".{os.getpid()}.tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
