"""Per-kernel gfx950 ISA comparison of two built libraries (no GPU needed).

    python scripts/isa_diff.py montecarlopathtracer_amd/lib/libmcpt_base.so montecarlopathtracer_amd/lib/libmcpt.so

Extracts the code objects of each library's .hip_fatbin (as
tests/test_kernel_resources.py does), disassembles them and compares every
kernel's instruction stream with addresses and branch offsets stripped.  Used
to show that a source cleanup leaves the shipped kernels' code unchanged.
"""
import os
import re
import subprocess
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_kernel_resources import LLVM, _code_objects, _kernels  # noqa: E402


def kernel_text(lib):
    out, res = {}, {}
    with tempfile.TemporaryDirectory() as td:
        for co in _code_objects(lib, Path(td)):
            res.update(_kernels(co))
            txt = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn",
                                  "--no-leading-addr", str(co)], check=True, capture_output=True, text=True).stdout
            cur = None
            for line in txt.splitlines():
                m = re.match(r"^(\S+):$", line.strip()) if line and not line.startswith((" ", "\t")) else None
                if m or re.match(r"^[0-9a-f]* ?<?(\S+?)>?:$", line.strip()):
                    name = (m.group(1) if m else re.match(r"^[0-9a-f]* ?<?(\S+?)>?:$", line.strip()).group(1))
                    cur = name.strip("<>")
                    out.setdefault(cur, [])
                    continue
                if cur and line.strip():
                    ins = re.sub(r"//.*$", "", line).strip()
                    ins = re.sub(r"<[^>]*>", "<L>", ins)
                    ins = re.sub(r"\b0x[0-9a-f]+\b", "#", ins) if ins.startswith(("s_cbranch", "s_branch")) else ins
                    if ins:
                        out[cur].append(ins)
    return out, res


def main(a, b):
    ka, ra = kernel_text(a)
    kb, rb = kernel_text(b)
    names = sorted(set(ra) | set(rb))
    same = 0
    for n in names:
        if n not in ra or n not in rb:
            print(f"{'only in ' + ('A' if n in ra else 'B'):10s} {n}")
            continue
        ta, tb = ka.get(n, []), kb.get(n, [])
        if ta == tb:
            same += 1
        else:
            print(f"differs    {n}: {len(ta)} vs {len(tb)} instructions, {ra[n]} vs {rb[n]}")
    print(f"{same} of {len(names)} kernels identical")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
