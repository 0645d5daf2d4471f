#!/usr/bin/env python3
"""The current-lines table of DESIGN.md §8 from bench records (one JSON line
each: a BENCH_rNN.json driver record's `parsed`, or a bench.py jsonl), every
cell citing the file it comes from.
usage: current_lines.py RECORD [SHARD_PROBE.txt]"""
import json
import os
import re
import sys


def load(path):
    if path.endswith(".json"):
        d = json.load(open(path))
        if "parsed" in d:
            ln = d["parsed"]
            # the driver keeps extra keys under extra_keys; the tail holds the full line
            tail = d.get("tail", "")
            for t in tail.splitlines():
                if t.startswith("{") and '"metric"' in t:
                    try:
                        ln = json.loads(t)
                    except json.JSONDecodeError:
                        pass
            return ln
        return d
    return [json.loads(x) for x in open(path) if x.startswith("{")][-1]


def row(name, ln, src):
    r = ln.get("roofline") or {}
    v = r.get("valu") or {}
    sched = (ln.get("config") or {}).get("schedule") or {}
    rs = r.get("read_split") or {}
    return (f"| {name} | {ln['value'] / 1e3:.2f} | {ln['ms_per_step']:.1f} | {r.get('frac')} | "
            f"{r.get('binding', '-')} {r.get('binding_frac', '')} | {v.get('useful_lane_frac', '-')} | "
            f"{rs.get('record_GB', '-')} | {sched.get('workspace_GB', '-')} | `{src}` |")


def main(rec, probe=None):
    ln = load(rec)
    src = os.path.relpath(rec)
    print("| config | G rays/s | ms/frame | extend HBM frac | binding roof | VALU useful lanes | "
          "reads past L2 beyond the ray stream, GB/frame | workspace GB | record |")
    print("|---|---|---|---|---|---|---|---|---|")
    print(row("C2 (1024², 1024 spp, wavefront)", ln, src))
    alt = ln.get("other_pipeline") or {}
    if alt.get("value"):
        print(f"| C2 megakernel | {alt['value'] / 1e3:.2f} | {alt['ms_per_step']:.1f} | - | - | - | - | - | `{src}` |")
    for k, name in (("c4", "C4 (70 k-tri mesh, 1024 spp)"), ("c5", "C5 (4096 spp, one GPU)")):
        x = (ln.get("extra_lines") or {}).get(k)
        if x and "value" in x:
            print(row(name, x, src + f" extra_lines.{k}"))
    if probe:
        shares = {}
        for t in open(probe):
            m = re.match(r"N=(\d+) wavefront streams=\d+ batch=\d+: ([0-9.]+) ms", t)
            if m:
                shares[int(m.group(1))] = float(m.group(2))
        if shares:
            frame = ln["ms_per_step"]
            cells = ", ".join(f"N = {n}: {ms:.1f} ms ({frame / n / ms * 100:.0f}% of 1/N)" for n, ms in
                              sorted(shares.items()))
            print(f"\nOne rank's C2 share (wavefront, `{os.path.relpath(probe)}`): {cells}.")


if __name__ == "__main__":
    main(*sys.argv[1:])
