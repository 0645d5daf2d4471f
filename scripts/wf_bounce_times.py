#!/usr/bin/env python3
"""Per-bounce extend / shade times from a rocprofv3 kernel trace of wavefront
renders on ONE stream (kernels serialized): dispatches are grouped per batch
(wf_generate starts one) and indexed by bounce.  usage: wf_bounce_times.py DIR"""
import csv
import glob
import sys
from collections import defaultdict


def main(d):
    rows = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    ext, sh = defaultdict(list), defaultdict(list)
    b_ext = b_sh = -1
    batches = 0
    for t0, t1, name in rows:
        if "wf_generate" in name:
            b_ext = b_sh = -1
            batches += 1
        elif "wf_extend" in name:
            b_ext += 1
            ext[b_ext].append((t1 - t0) / 1e6)
        elif "wf_shade" in name:
            b_sh += 1
            sh[b_sh].append((t1 - t0) / 1e6)
    print(f"batches {batches}")
    for b in sorted(ext):
        e, s = ext[b], sh.get(b, [0])
        print(f"bounce {b}: extend {sum(e) / batches:8.2f} ms/frame-batch-avg x{len(e)}  "
              f"(per dispatch {sum(e) / len(e):.3f})  shade {sum(s) / max(len(s), 1):.3f}")
    print("extend total per batch", sum(sum(v) for v in ext.values()) / batches)


if __name__ == "__main__":
    main(sys.argv[1])
