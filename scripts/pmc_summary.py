#!/usr/bin/env python3
"""Fold the rocprofv3 passes of scripts/profile_round.sh into one JSON summary.

Per-launch values of the path kernel (the dominant kernel): counters summed
over XCDs/SEs by rocprofv3's csv (one row per dispatch x counter).  Derived
numbers follow MI355X_MICROARCH.md: FETCH_SIZE doubled (gfx950 streaming-read
undercount), SQ_*CYCLES in quad-cycles, clock = GRBM_GUI_ACTIVE / 8 / wall.
"""
import csv
import glob
import json
import os
import sys

MATCH = os.environ.get("KERNEL_MATCH", "path_kernel")
# bench.py times the lean megakernel (last template argument COUNT = false) and
# runs the counting one once, untimed: profile the lean one
LEAN = os.environ.get("KERNEL_MATCH_LEAN", "false>(mcpt::KernelParams)")


def _pick(name):
    return MATCH in name and (not LEAN or name.endswith(LEAN))


def read_counters(d):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if not _pick(row.get("Kernel_Name", "")):
                    continue
                k = row["Counter_Name"]
                vals.setdefault(k, {}).setdefault(row["Dispatch_Id"], 0.0)
                vals[k][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in vals.items()}


def main(out):
    per = {}
    for sub in sorted(os.listdir(out)):
        p = os.path.join(out, sub)
        if os.path.isdir(p) and sub != "kt":
            for k, v in read_counters(p).items():
                per.setdefault(k, v)
    bench = None
    bj = os.path.join(out, "bench.jsonl")
    if os.path.exists(bj):
        for line in open(bj):
            if line.startswith("{"):
                bench = json.loads(line)
    kstats = None
    for f in glob.glob(os.path.join(out, "kt", "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if _pick(row["Name"]):
                    kstats = {"name": row["Name"], "calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"])}
    d = {}
    rays = bench["rays_per_step"] if bench else None
    g = per.get
    if g("FETCH_SIZE") is not None:
        d["hbm_read_GB_corrected_x2"] = 2 * g("FETCH_SIZE") * 1024 / 1e9
    if g("WRITE_SIZE") is not None:
        d["hbm_write_GB"] = g("WRITE_SIZE") * 1024 / 1e9
    if rays:
        for k, name in (("SQ_INSTS_VALU", "valu_wave_instr_per_ray"), ("SQ_INSTS_SALU", "salu_per_ray"),
                        ("SQ_INSTS_LDS", "lds_instr_per_ray"), ("SQ_INSTS_BRANCH", "branch_per_ray"),
                        ("SQ_INSTS_VALU_FLOPS_FP64", "fp64_flops_per_ray"),
                        ("SQ_INSTS_VALU_TRANS_F32", "trans_f32_per_ray")):
            if g(k) is not None:
                d[name] = g(k) / rays
    if g("SQ_THREAD_CYCLES_VALU") and g("SQ_ACTIVE_INST_VALU"):
        d["valu_lane_utilisation"] = g("SQ_THREAD_CYCLES_VALU") / (64.0 * g("SQ_ACTIVE_INST_VALU"))
    if g("SQ_WAVE_CYCLES"):
        wc = g("SQ_WAVE_CYCLES")
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS"):
            if g(k) is not None:
                d["frac_wave_cycles_" + k[3:].lower()] = g(k) / wc
    if g("SQ_LDS_BANK_CONFLICT") and g("SQ_INSTS_LDS"):
        d["lds_bank_conflict_cycles_per_lds_instr"] = g("SQ_LDS_BANK_CONFLICT") / g("SQ_INSTS_LDS")
    if g("TCC_HIT") is not None and g("TCC_MISS") is not None:
        d["l2_hit_rate"] = g("TCC_HIT") / max(g("TCC_HIT") + g("TCC_MISS"), 1.0)
        d["l2_requests_GB_x128B"] = (g("TCC_HIT") + g("TCC_MISS")) * 128 / 1e9
    if g("TCP_TOTAL_CACHE_ACCESSES") and g("TCP_TCC_READ_REQ") is not None:
        d["l1_miss_to_l2_frac"] = g("TCP_TCC_READ_REQ") / g("TCP_TOTAL_CACHE_ACCESSES")
    if g("GRBM_GUI_ACTIVE") and kstats:
        d["effective_clock_GHz"] = g("GRBM_GUI_ACTIVE") / 8 / kstats["avg_ns"]
    print(json.dumps({"kernel": kstats, "per_launch_counters": per, "derived": d, "bench_line": bench}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
