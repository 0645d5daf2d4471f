#!/usr/bin/env python3
"""Recompute a bench line's wf_extend roofline from the raw rocprofv3 PMC csv it
kept (bench.py --keep-pmc DIR; committed under profiles/rNN/pmc_wf):
achieved = (2 x FETCH_SIZE + WRITE_SIZE) KiB of the extend dispatches / their
summed duration in the FETCH_SIZE pass, frac = achieved / 8000 GB/s; with the
bench line (its per-ray counts, rays per frame and the CU count it ran on) also
roofline.lds from the wf_lds pass and roofline.binding_frac (max of the HBM,
LDS-array and VALU-issue fractions; the VALU figure from the wf_valu pass).
With a wf_req pass (TCC_EA0_RDREQ by request size) also the exact fabric read
bytes, FETCH_SIZE's factor for this pattern, and the ray-stream / record split.
usage: roofline_from_csv.py profiles/r05/pmc_wf [profiles/r05/bench.jsonl] [CUs=256] [c4|c5]
       (c4 / c5: the bench line's extra line of that name, with DIR its pmc_wf/c4 csv)"""
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(d, line=None, cus=256, extra=None):
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    f = b.read_wf_kernels(os.path.join(d, "wf_fetch"))["extend"]
    w = b.read_wf_kernels(os.path.join(d, "wf_write"))["extend"]
    rd, wr = 2.0 * f["FETCH_SIZE"] * 1024.0, w["WRITE_SIZE"] * 1024.0
    gbs = (rd + wr) / f["ns"]
    out = {"extend_read_GB": round(rd / 1e9, 3), "extend_write_GB": round(wr / 1e9, 3), "ms": round(f["ns"] / 1e6, 3),
           "launches": f["dispatches"], "achieved_GBps": round(gbs, 2), "frac": round(gbs / b.HBM_PEAK_GBS, 5)}
    qd = os.path.join(d, "wf_req")
    if os.path.isdir(qd):   # exact fabric reads by request size (the FETCH_SIZE calibration)
        q = b.read_wf_kernels(qd)["extend"]
        exact = 32.0 * q.get("TCC_EA0_RDREQ_32B", 0) + 64.0 * q.get("TCC_EA0_RDREQ_64B", 0) + \
            128.0 * q["TCC_EA0_RDREQ_128B"]
        out["exact_read_GB"] = round(exact / 1e9, 3)
        out["fetch_size_factor"] = round(exact / (f["FETCH_SIZE"] * 1024.0), 4)
    if line:
        ln = [json.loads(x) for x in open(line) if x.startswith("{")][-1]
        if extra:   # e.g. c4: the line's extra line of that name
            ln = ln["extra_lines"][extra]
        r = ln["roofline"]
        if "exact_read_GB" in out:
            rays = ln["rays_per_step"] / ln["n_gpus"]
            paths = ln["paths_per_step"] / ln["n_gpus"]
            ray_gb = b.ray_stream_bytes(rays, paths, ln["config"].get("kernel_variant")) / 1e9
            out["ray_GB"], out["record_GB"] = round(ray_gb, 3), round(out["exact_read_GB"] - ray_gb, 3)
        out["bench_line"] = {"achieved": r["achieved"], "frac": r["frac"], "traffic": r["traffic"],
                             "read_split": r.get("read_split")}
        cus = int(cus)
        roof = {"frac": out["frac"]}
        vd = os.path.join(d, "wf_valu")
        if os.path.isdir(vd):
            v = b.read_wf_kernels(vd)["extend"]
            roof["valu"] = b.valu_block(v, cus, v["ns"] / 1e6, ln["rays_per_step"] / ln["n_gpus"])
        ldd = os.path.join(d, "wf_lds")
        if os.path.isdir(ldd) and ln["config"].get("kernel_variant") == 4:   # scene image in LDS
            lc = b.read_wf_kernels(ldd)["extend"]
            pr = r["algorithmic"]["per_ray"]
            rays = ln["rays_per_step"] / ln["n_gpus"]
            roof["lds"] = b.lds_block(lc, cus, {k: pr[k] * rays for k in ("inner_visits", "leaf_refs", "tri_tests")})
            out["lds"] = roof["lds"]
            out["bench_line"]["lds"] = r.get("lds")
        out.update(b.binding_of(roof))
        out["bench_line"]["binding_frac"] = r.get("binding_frac")
        out["bench_line"]["binding"] = r.get("binding")
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:])
