#!/usr/bin/env python3
"""Per wavefront kernel (lean extend, bounce-0 extend, shade, generate): the
SQ counters of scripts/pmc_extend_stalls.sh summed over one render's
dispatches, as fractions of SQ_WAVE_CYCLES (all SQ_*CYCLES count quad-cycles;
WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES, MI355X_MICROARCH.md
'rocprofv3 PMC slots') and instructions per wave.  usage: stall_summary.py DIR"""
import csv
import glob
import json
import os
import sys

CUS = 256
KINDS = (("wf_extend_primary", "extend_bounce0"), ("wf_extend<", "extend"), ("wf_shade", "shade"),
         ("wf_generate", "generate"))


def kind(name):
    if "true>(mcpt" in name and "wf_extend" in name:   # the counting (untimed) variants
        return None
    return next((k for key, k in KINDS if key in name), None)


def main(d):
    acc, ns, src = {}, {}, {}
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        for row in csv.DictReader(open(f)):
            k = kind(row.get("Kernel_Name", ""))
            if k is None:
                continue
            cn = row["Counter_Name"]
            if src.setdefault(cn, f) != f:   # a counter collected in two passes: count one
                continue
            c = acc.setdefault(k, {})
            c[cn] = c.get(cn, 0.0) + float(row["Counter_Value"])
            if row["Counter_Name"] == "SQ_WAVE_CYCLES":
                ns.setdefault(k, {})[row["Dispatch_Id"]] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    out = {}
    for k, c in acc.items():
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        r = {"ms": round(sum(ns.get(k, {}).values()) / 1e6, 2)}
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_MISC",
                      "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_FLAT"):
                if n in c:
                    r["frac_" + n[3:].lower()] = round(c[n] / wc, 4)
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM",
                  "SQ_INSTS_SMEM"):
            if n in c:
                r[n[3:].lower() + "_G"] = round(c[n] / 1e9, 3)
        if c.get("SQ_THREAD_CYCLES_VALU") and c.get("SQ_INSTS_VALU"):
            r["lane_use_per_valu_inst"] = round(c["SQ_THREAD_CYCLES_VALU"] / 64.0 / c["SQ_INSTS_VALU"], 4)
        if c.get("SQ_LDS_BANK_CONFLICT") and c.get("SQ_INSTS_LDS"):
            r["lds_conflict_cycles_per_lds_inst"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"], 3)
        if c.get("SQ_LDS_IDX_ACTIVE") and c.get("GRBM_GUI_ACTIVE"):
            # LDS-array cycles summed over CUs / (CUs x kernel cycles); GRBM_GUI_ACTIVE is summed over 8 XCDs
            r["lds_idx_active_G"] = round(c["SQ_LDS_IDX_ACTIVE"] / 1e9, 3)
            r["lds_array_busy"] = round(c["SQ_LDS_IDX_ACTIVE"] / CUS / (c["GRBM_GUI_ACTIVE"] / 8), 4)
        if c.get("GRBM_GUI_ACTIVE") and r["ms"]:
            r["clock_GHz"] = round(c["GRBM_GUI_ACTIVE"] / 8 / (r["ms"] * 1e6), 3)
        out[k] = r
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
