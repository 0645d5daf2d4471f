"""Compile tests/cpp/pw_tracer_dropin.cpp against include/ and libmcpt.so (test infrastructure)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "_build", "pw_tracer_dropin")


def build():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    libdir = os.path.join(ROOT, "montecarlopathtracer_amd", "lib")
    subprocess.run(["g++", "-std=c++17", "-O1", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(HERE, "pw_tracer_dropin.cpp"), "-L" + libdir, "-lmcpt",
                    "-Wl,-rpath," + libdir, "-Wl,--allow-shlib-undefined", "-o", OUT], check=True)
    return OUT


if __name__ == "__main__":
    print(build())
