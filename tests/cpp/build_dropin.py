"""Compile the C++ adapter test programs in tests/cpp/ against include/ (test infrastructure).

pw_tracer_dropin  include/mcpt_pw_tracer.hpp: the CVMCTracer main.cpp call sequence
qe_viewer         include/mcpt_qe_viewer.hpp: the QuinEngine OnUpdate frame loop
image_io          include/mcpt_image_io.hpp: the main.cpp:19-29 encode, PNG and PFM
half_box_probe    csrc/half_box.hpp: the outward-rounded fp16 leaf boxes (vs the oracle's)
fastdiv_probe     csrc/render_launch.hpp FastDiv: multiply-high division == n / d
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
LINKS_MCPT = {"pw_tracer_dropin": True, "qe_viewer": True, "image_io": False, "half_box_probe": False,
              "fastdiv_probe": False}


def build(name: str = "pw_tracer_dropin") -> str:
    out = os.path.join(HERE, "_build", name)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-I" + os.path.join(ROOT, "include"), os.path.join(HERE, name + ".cpp")]
    if name == "fastdiv_probe":   # includes a device header: HIP's host-side declarations
        cmd += ["-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
    if LINKS_MCPT[name]:
        libdir = os.path.join(ROOT, "montecarlopathtracer_amd", "lib")
        cmd += ["-L" + libdir, "-lmcpt", "-Wl,-rpath," + libdir, "-Wl,--allow-shlib-undefined"]
    subprocess.run(cmd + ["-o", out], check=True)
    return out


if __name__ == "__main__":
    for n in LINKS_MCPT:
        print(build(n))
