"""Static instruction count of each phase of the extend kernels (diagnostic,
no GPU): compile wavefront.hip with -DMCPT_PHASE_MARKERS (trace_device.hpp
MCPT_MARK: `s_nop 15; s_nop n` at the phase boundaries), disassemble, and
count the instructions of each region that follows marker n, by class.

  python scripts/phase_isa.py [obj]     (default: builds /tmp/mcpt_wf_mark.o)

Markers: 1 descent step (one copy per unrolled step), 2 leaf reached,
3 leaf call (stack-top read ahead + the triangle pair), 4 pop, 5 burst
iteration head (until the traversal call), 6 burst loop tail (ballots,
exit test), 7 hand-off, 8 after the hand-off (loop exit test).
"""
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter, defaultdict
from pathlib import Path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "montecarlopathtracer_amd"))
from test_kernel_resources import LLVM, _code_objects  # noqa: E402

KERNELS = {"lds lean": r"wf_extendILi1ELi4ELi1024ELb0ELb0E", "global lean": r"wf_extendILi0ELi\d+ELi256ELb0ELb0E"}


def build(out):
    import _build as B
    cmd = [B._hipcc(), "-x", "hip", "--offload-arch=gfx950", "-mllvm", "-amdgpu-sched-strategy=max-ilp"] + \
        B.COMMON + B.SOURCE_FLAGS["wavefront.hip"] + ["-DMCPT_PHASE_MARKERS", "-c",
                                                      os.path.join(B.CSRC, "wavefront.hip"), "-o", out]
    subprocess.run(cmd, check=True, capture_output=True)
    return out


def disasm(obj):
    """kernel -> [(offset, instruction, branch target offset or None)]"""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for co in _code_objects(obj, Path(td)):
            txt = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", str(co)],
                                 check=True, capture_output=True, text=True).stdout
            cur, base = None, None
            for line in txt.splitlines():
                m = re.match(r"^([0-9a-f]+) <(\S+)>:$", line.strip())
                if m:
                    cur, base = m.group(2), int(m.group(1), 16)
                    out[cur] = []
                elif cur and line.strip() and not line.strip().startswith(";"):
                    a = re.search(r"//\s*([0-9A-Fa-f]+):", line)
                    t = re.search(r"<[^>]*\+0x([0-9a-f]+)>", line)
                    out[cur].append((int(a.group(1), 16) - base if a else None, re.sub(r"\s*//.*$", "", line.strip()),
                                     int(t.group(1), 16) if t else None))
    return out


def klass(ins):
    op = ins.split()[0]
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    return "salu"


def regions(ins):
    """marker id -> list of per-copy Counters of the instructions until the next
    marker; class + "_c" for instructions inside a forward s_cbranch_execz
    region opened within the phase (skipped when no lane of the wave takes
    that side)"""
    res = defaultdict(list)
    cur, cnt, i = None, None, 0
    guard_end = []          # end offsets of the enclosing execz-skippable regions
    while i < len(ins):
        off, txt, tgt = ins[i]
        guard_end = [e for e in guard_end if off is None or off < e]
        if txt == "s_nop 15" and i + 1 < len(ins) and ins[i + 1][1].startswith("s_nop "):
            if cur is not None:
                res[cur].append(cnt)
            cur, cnt = int(ins[i + 1][1].split()[1]), Counter()
            guard_end = []          # (only regions opened inside this phase count)
            i += 2
            continue
        if txt.startswith("s_cbranch_execz") and tgt is not None and off is not None and tgt > off:
            guard_end.append(tgt)
        if cur is not None:
            cnt[klass(txt) + ("_c" if guard_end else "")] += 1
            cnt[klass(txt) + f"_d{min(len(guard_end), 2)}"] += 1
        i += 1
    if cur is not None:
        res[cur].append(cnt)
    return res


def main():
    obj = sys.argv[1] if len(sys.argv) > 1 else build("/tmp/mcpt_wf_mark.o")
    d = disasm(obj)
    for label, pat in KERNELS.items():
        names = [n for n in d if re.search(pat, n)]
        if len(names) != 1:
            print(label, "not found", names)
            continue
        ins = d[names[0]]
        print(f"== {label}: {len(ins)} instructions ({names[0][:60]})")
        for m, copies in sorted(regions(ins).items()):
            tot = Counter()
            for c in copies:
                tot.update(c)
            n = len(copies)
            print(f"  marker {m}: {n} cop{'y' if n == 1 else 'ies'}, per copy: " +
                  " ".join(f"{k} {tot[k] / n:.1f}+{tot[k + '_c'] / n:.1f}" for k in ("valu", "salu", "lds", "vmem")) +
                  "  (always + inside execz-skippable regions); valu by nesting 0/1/2+: " +
                  "/".join(f"{tot['valu_d' + str(i)] / n:.1f}" for i in range(3)))


if __name__ == "__main__":
    main()
