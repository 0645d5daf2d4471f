#!/usr/bin/env python3
"""Recompute a bench line's wf_extend roofline from the raw rocprofv3 PMC csv it
kept (bench.py --keep-pmc DIR; committed under profiles/rNN/pmc_wf):
achieved = (2 x FETCH_SIZE + WRITE_SIZE) KiB of the extend dispatches / their
summed duration in the FETCH_SIZE pass, frac = achieved / 8000 GB/s.
usage: roofline_from_csv.py profiles/r03/pmc_wf [profiles/r03/bench.jsonl]"""
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(d, line=None):
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    f = b.read_wf_kernels(os.path.join(d, "wf_fetch"))["extend"]
    w = b.read_wf_kernels(os.path.join(d, "wf_write"))["extend"]
    rd, wr = 2.0 * f["FETCH_SIZE"] * 1024.0, w["WRITE_SIZE"] * 1024.0
    gbs = (rd + wr) / f["ns"]
    out = {"extend_read_GB": round(rd / 1e9, 3), "extend_write_GB": round(wr / 1e9, 3), "ms": round(f["ns"] / 1e6, 3),
           "launches": f["dispatches"], "achieved_GBps": round(gbs, 2), "frac": round(gbs / b.HBM_PEAK_GBS, 5)}
    if line:
        r = [json.loads(x) for x in open(line) if x.startswith("{")][-1]["roofline"]
        out["bench_line"] = {"achieved": r["achieved"], "frac": r["frac"], "traffic": r["traffic"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:])
