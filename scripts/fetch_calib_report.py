#!/usr/bin/env python3
"""Report of scripts/fetch_calib.sh: the L2 fabric-read counters against known
byte counts, and the same counters over one C4 frame's wf_extend.

Passes (one rocprofv3 --pmc run each; csv under DIR/calib_pN, DIR/c4_pN):
  p1 FETCH_SIZE                         (rocprofv3's derived KiB)
  p2 TCC_EA0_RDREQ{,_32B,_64B,_128B}    (requests by size: exact bytes =
                                         32 x n32 + 64 x n64 + 128 x n128)
  p3 TCC_EA0_RDREQ_DRAM{,_32B} TCC_BUBBLE (DRAM share in 32-B units)
  p4 WRITE_SIZE
  p5 TCC_EA0_WRREQ{,_64B} TCC_EA0_WR_UNCACHED_32B TCC_EA0_WRREQ_WRITE_DRAM_32B
usage: fetch_calib_report.py DIR [c4 bench line .jsonl (rays / paths per frame)]
"""
import csv
import glob
import json
import os
import sys

KNOWN = {   # kernel -> (label, known bytes given the records count n)
    "calib_stream": ("stream 1 GiB, 16 B/lane", lambda n: 1 << 30),
    "calib_gather<128, 0>": ("48-B records, one per 128-B line, offset 0", lambda n: 4 * n + 48 * n),
    "calib_gather<128, 40>": ("48-B records, one per 128-B line, offset 40", lambda n: 4 * n + 48 * n),
    "calib_gather<48, 0>": ("packed 48-B records (C4 pair-record layout)", lambda n: 4 * n + 48 * n),
}


def read(d, match):
    """counter -> value summed over the dispatches of kernels whose name contains `match`"""
    vals, ns = {}, {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if match not in row.get("Kernel_Name", ""):
                    continue
                vals[row["Counter_Name"]] = vals.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
                ns[row["Dispatch_Id"]] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    vals["ns"] = sum(ns.values())
    vals["dispatches"] = len(ns)
    return vals


def bytes_of(d, prefix, match):
    c = {}
    for i in range(1, 6):
        p = os.path.join(d, f"{prefix}_p{i}")
        if os.path.isdir(p):
            for k, v in read(p, match).items():
                c.setdefault(k, v)
    g = lambda k: c.get(k)  # noqa: E731
    out = {"counters": {k: v for k, v in c.items() if k not in ("ns", "dispatches")}}
    if g("FETCH_SIZE") is not None:
        out["fetch_size_B"] = g("FETCH_SIZE") * 1024.0
    if g("TCC_EA0_RDREQ_32B") is not None and g("TCC_EA0_RDREQ_64B") is not None:
        n128 = g("TCC_EA0_RDREQ_128B") or 0.0
        out["read_exact_B"] = 32.0 * g("TCC_EA0_RDREQ_32B") + 64.0 * g("TCC_EA0_RDREQ_64B") + 128.0 * n128
        out["requests"] = {"32B": g("TCC_EA0_RDREQ_32B"), "64B": g("TCC_EA0_RDREQ_64B"), "128B": n128,
                           "all": g("TCC_EA0_RDREQ")}
    if g("TCC_EA0_RDREQ_DRAM_32B") is not None:
        out["read_dram_B"] = 32.0 * g("TCC_EA0_RDREQ_DRAM_32B")
    if g("WRITE_SIZE") is not None:
        out["write_size_B"] = g("WRITE_SIZE") * 1024.0
    if g("TCC_EA0_WRREQ") is not None and g("TCC_EA0_WRREQ_64B") is not None:
        out["write_exact_B"] = 32.0 * (g("TCC_EA0_WRREQ") - g("TCC_EA0_WRREQ_64B")) + 64.0 * g("TCC_EA0_WRREQ_64B")
        if g("TCC_EA0_WR_UNCACHED_32B") is not None:
            out["write_uncached_B"] = 32.0 * g("TCC_EA0_WR_UNCACHED_32B")
        if g("TCC_EA0_WRREQ_WRITE_DRAM_32B") is not None:
            out["write_dram_B"] = 32.0 * g("TCC_EA0_WRREQ_WRITE_DRAM_32B")
    return out


def main(d, c4line=None):
    info = {}
    for ln in open(os.path.join(d, "calib_p1.log")):
        if ln.startswith("{"):
            info = json.loads(ln)
    n = info.get("records", 1 << 20)
    rep = {"records": n, "calibration": {}, "c4_extend": None}
    for k, (label, known) in KNOWN.items():
        b = bytes_of(d, "calib", k)
        kb = known(n)
        r = {"label": label, "known_B": kb}
        for key in ("fetch_size_B", "read_exact_B", "read_dram_B"):
            if key in b:
                r[key] = b[key]
                r[key.replace("_B", "_over_known")] = round(b[key] / kb, 4)
        if "fetch_size_B" in b and "read_exact_B" in b:
            r["exact_over_fetch_size"] = round(b["read_exact_B"] / b["fetch_size_B"], 4)
        r["requests"] = b.get("requests")
        rep["calibration"][k] = r
    c4 = bytes_of(d, "c4", "wf_extend")
    if c4:
        out = {k: round(v / 1e9, 3) for k, v in c4.items() if k.endswith("_B")}
        out = {k[:-2] + "_GB": v for k, v in out.items()}
        if "fetch_size_B" in c4 and "read_exact_B" in c4:
            out["exact_over_fetch_size"] = round(c4["read_exact_B"] / c4["fetch_size_B"], 4)
        out["requests"] = c4.get("requests")
        out["write_counters"] = {k: v for k, v in c4["counters"].items() if "WR" in k}
        if c4line and os.path.exists(c4line):
            ln = [json.loads(x) for x in open(c4line) if x.startswith("{")][-1]
            ln = (ln.get("extra_lines") or {}).get("c4", ln)   # the C4 line of a default bench line
            rays, paths = ln["rays_per_step"], ln["paths_per_step"]
            # the extend's ray stream: bounce 0 reads 16 B (direction; the origin is the eye), later
            # bounces 32 B (origin + direction); it writes a 4-B hit id per ray
            ray_rd = 16.0 * paths + 32.0 * (rays - paths)
            out["ray_stream_read_GB"] = round(ray_rd / 1e9, 3)
            out["hit_id_write_GB"] = round(4.0 * rays / 1e9, 3)
            if "read_exact_B" in c4:
                out["record_read_GB"] = round((c4["read_exact_B"] - ray_rd) / 1e9, 3)
        rep["c4_extend"] = out
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
