#!/usr/bin/env python3
"""Timeline of the last frame in a rocprofv3 --kernel-trace csv of a
multi-stream wavefront render: busy union, gaps, and how long extends ran
with nothing beside them.  usage: frame_timeline.py <dir> [frames=4]
(the last `frames`-th part of the generate launches starts the last frame)."""
import csv
import glob
import re
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))


def nm(s):
    m = re.search(r"(wf_\w+|reduce_kernel|path_kernel|rocclr_\w+)", s)
    return m.group(1) if m else s[:20]


ev = [(nm(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
ev = [e for e in ev if not e[0].startswith("rocclr")]
red = [k for k, e in enumerate(ev) if e[0] == "reduce_kernel"]
# last frame: after the second-to-last reduce
a = red[-2] + 1 if len(red) >= 2 else 0
fr = ev[a:red[-1] + 1]
t0, t1 = fr[0][1], fr[-1][2]
print(f"frame {(t1 - t0) / 1e6:.2f} ms, {len(fr)} kernels")
# busy union and per-type coverage
pts = sorted([(s, 1, n) for n, s, e in fr] + [(e, -1, n) for n, s, e in fr])
active = {}
busy = ext_alone = ext_any = 0
last = t0
for t, d, n in pts:
    dt = t - last
    kinds = [k for k, c in active.items() if c > 0]
    if kinds:
        busy += dt
    if any(k.startswith("wf_extend") for k in kinds):
        ext_any += dt
        if len(kinds) == 1 and sum(active.values()) == 1:
            ext_alone += dt
    active[n] = active.get(n, 0) + d
    last = t
span = t1 - t0
print(f"busy {busy / 1e6:.2f} ms ({busy / span:.1%}), an extend running {ext_any / 1e6:.2f} ms "
      f"({ext_any / span:.1%}), one extend alone {ext_alone / 1e6:.2f} ms")
print("first 12:", " ".join(f"{n[3:9]}@{(s - t0) / 1e3:.0f}-{(e - t0) / 1e3:.0f}" for n, s, e in fr[:12]))
print("last 12:", " ".join(f"{n[3:9]}@{(s - t0) / 1e3:.0f}-{(e - t0) / 1e3:.0f}" for n, s, e in fr[-12:]))
