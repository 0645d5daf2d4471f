#!/usr/bin/env python3
"""bench.py -- Cornell Box 1024x1024 @ 1024 spp on N MI355X (BASELINE.json configs[1]/[2]).

One step = one full path-traced frame of the workload (every pixel, every
sample, up to 7 scatter events + 1 terminal query per path) through the C ABI
(mcpt_render_device) -- by default on the wavefront pipeline, whose image is
bit-identical to the megakernel's and which is the faster of the two on
MI355X (N = 1 runs also time the megakernel, reported under other_pipeline)
-- plus, for N > 1, the RCCL gather of the per-rank
tile buffers to rank 0 and its unpermute into the image.  Pixels are sharded
as interleaved 8x8 tiles (tile t -> rank t % N); total work is fixed, so the
scaling is strong.  value = closest-hit queries of all ranks / max-over-ranks
wall time (Mray/s).

Roofline: `achieved` = the MEASURED HBM bytes of the frame's kernels (rocprofv3
PMC passes of this build and workload, run by this bench in child processes:
FETCH_SIZE x2 + WRITE_SIZE) / their HIP-event duration; the traversal (path
kernel / wavefront extend) is bound by VALU issue and latency, reported under
roofline.valu (issue and lane fractions from the same passes); SURVEY.md
section 8(d)'s algorithmic bytes (LDS/L2-served) are reported separately
under roofline.algorithmic.  Wavefront runs report each
kernel's measured HBM traffic and rate under roofline.kernels (the queue
streams: SURVEY 8(f)1), and every N = 1 run measures a 1 GiB device copy as
the roofline's second denominator (roofline.peak_copy_measured).  cpu_baseline = BASELINE
configs[0] (C1: 512x512, 16 spp, whole frame, one thread) on the CPU oracle,
plus the same oracle on all of this process's cores over whole frames of the
workload at a few samples per pixel.

Launch:  python bench.py [--gpus 1 --steps 3 --warmup 1]
         python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
             --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...
         python bench.py --gpus N ...   (no launcher: starts the line above as a
             child process; fewer than N visible GPUs exits non-zero)
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mray/s + achieved HBM GB/s, Cornell Box 1024spp at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def algorithmic_bytes(st: dict, pixels: int) -> dict:
    """B_ray = 32*N_node + 4*N_leafref + 48*N_tri + 96*N_shade, + 16 B per pixel.
    'own' = the same counts priced with this kernel's records (8-B KD nodes)."""
    nodes = st["inner_visits"] + st["leaf_visits"]
    survey = 32 * nodes + 4 * st["leaf_refs"] + 48 * st["tri_tests"] + 96 * st["shades"] + 16 * pixels
    own = 8 * nodes + 4 * st["leaf_refs"] + 48 * st["tri_tests"] + 96 * st["shades"] + 16 * pixels
    return {"survey": survey, "own": own}


def ray_stream_bytes(rays: float, paths: float, variant: int, qe: bool = False) -> float:
    """Bytes of ray stream the extend reads per frame (wavefront.hip implicit0 /
    the packet bounce 0): later bounces read 32 B per ray (origin + direction).
    Bounce 0 in CV mode reads 16 B per path (the direction; the origin is the
    eye), and nothing on the LDS wavefront (kernel variant 4), whose bounce-0
    packet extend computes the primary rays itself (MCPT_WF_GEN0); in
    QuinEngine mode (near-plane origins) bounce 0 reads both streams, 32 B per
    path.  The material sort (wf_sort) sorts inside the shade: same streams."""
    b0 = 32.0 if qe else (0.0 if variant == 4 else 16.0)
    return b0 * paths + 32.0 * (rays - paths)


def hit_write_bytes(rays: float) -> float:
    """The extend's hit stream: the 4-B triangle id per ray."""
    return 4.0 * rays


def _workload_args(args, shard=(1, 0)) -> list:
    return ["--scene", args.scene, "--width", str(args.width), "--height", str(args.height), "--spp", str(args.spp),
            "--spp-chunk", str(args.spp_chunk), "--pipeline", args.pipeline, "--wf-batch", str(args.wf_batch),
            "--wf-streams", str(args.wf_streams), "--pmc-shard", f"{shard[0]},{shard[1]}", "--layout", args.layout] + \
        [x for kv in args.set for x in ("--set", kv)] + (["--counting"] if args.counting else []) + \
        (["--wf-sort"] if args.wf_sort else []) + ["--kd-build", args.kd_build]


SCHED_FIELDS = ("wf_refill", "wf_group_shift", "ready_thresh", "tail_units_per_lane", "tail_units", "wf_mem_limit")


def _tuning(args) -> dict:
    out = {}
    for kv in args.set:
        k, _, v = kv.partition("=")
        if k not in SCHED_FIELDS:
            raise SystemExit(f"--set {kv}: field must be one of {SCHED_FIELDS}")
        out[k] = int(v)
    return out


WF_KERNELS = (("wf_extend", "extend"), ("wf_shade", "shade"), ("wf_generate", "generate"),
              ("wf_accumulate", "accumulate"))


def read_wf_kernels(d: str) -> dict:
    """Per wavefront kernel class, summed over its dispatches of one render:
    counter values and the dispatches' durations (ns) from the PMC csv."""
    import csv
    import glob
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                cls = next((c for key, c in WF_KERNELS if key in name), None)
                if cls is None:
                    continue
                k = out.setdefault(cls, {"ns": {}, "counters": {}})
                k["ns"][row["Dispatch_Id"]] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                cn = row["Counter_Name"]
                k["counters"][cn] = k["counters"].get(cn, 0.0) + float(row["Counter_Value"])
    return {c: {"ns": sum(v["ns"].values()), "dispatches": len(v["ns"]), **v["counters"]} for c, v in out.items()}


def pmc_pass(args, counters: list, tag: str, timeout_s: int = 150, reader=None, shard=(1, 0)) -> dict:
    """One rocprofv3 PMC pass over ONE render of the same workload, in a child
    process (MI355X_MICROARCH.md 'rocprofv3 PMC slots': one pass per counter
    group -- FETCH_SIZE uses 3 of the 4 TCC slots, WRITE_SIZE 2).  Returns the
    per-launch counter values of the timed path kernel, or {} if the pass fails."""
    import shutil
    import signal
    import subprocess
    import tempfile
    if not shutil.which("rocprofv3"):
        return {}
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from pmc_summary import read_counters
    out = tempfile.mkdtemp(prefix=f"mcpt_pmc_{tag}_", dir="/tmp")
    cmd = ["rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", out, "-o", "run", "--",
           sys.executable, os.path.abspath(__file__), "--pmc-child"] + _workload_args(args, shard)
    env = dict(os.environ, TMPDIR="/tmp")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    proc = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                            start_new_session=True)
    try:
        proc.wait(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        os.killpg(proc.pid, signal.SIGKILL)
        proc.wait()
        return {}
    try:
        vals = (reader or read_counters)(out) if proc.returncode == 0 else {}
        if args.keep_pmc and proc.returncode == 0:   # the raw csv behind the line, for profiles/
            import glob
            dst = os.path.join(args.keep_pmc, tag)
            os.makedirs(dst, exist_ok=True)
            for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
                shutil.copy(f, os.path.join(dst, os.path.basename(f)))
    finally:
        shutil.rmtree(out, ignore_errors=True)
    return vals


def live_counters(args) -> dict:
    """HBM bytes and VALU issue of the path kernel, measured now on this build
    (three separate passes, MI355X_MICROARCH.md HBM section: FETCH_SIZE doubled
    on gfx950, WRITE_SIZE exact; both in KiB)."""
    c = {}
    for tag, counters in (("fetch", ["FETCH_SIZE"]), ("write", ["WRITE_SIZE"]),
                          ("valu", ["SQ_INSTS_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU",
                                    "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"])):
        c.update(pmc_pass(args, counters, tag))
    return c


def wavefront_hbm(args, shard=(1, 0)) -> dict:
    """Measured HBM bytes and time of each wavefront kernel over one render
    (FETCH_SIZE doubled + WRITE_SIZE, as live_counters): the queue streams are
    where this pipeline meets the HBM roofline."""
    f = pmc_pass(args, ["FETCH_SIZE"], "wf_fetch", reader=read_wf_kernels, shard=shard)
    w = pmc_pass(args, ["WRITE_SIZE"], "wf_write", reader=read_wf_kernels, shard=shard)
    v = pmc_pass(args, ["SQ_INSTS_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES",
                        "GRBM_GUI_ACTIVE"], "wf_valu", reader=read_wf_kernels, shard=shard)
    ld = pmc_pass(args, ["SQ_INSTS_LDS", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT", "GRBM_GUI_ACTIVE"], "wf_lds",
                  reader=read_wf_kernels, shard=shard)
    # the L2's fabric read requests by size (FETCH_SIZE's inputs on gfx950): exact bytes
    # = 32 n32 + 64 n64 + 128 n128, the calibration of FETCH_SIZE x 2 for this access pattern
    rq = pmc_pass(args, ["TCC_EA0_RDREQ", "TCC_EA0_RDREQ_32B", "TCC_EA0_RDREQ_64B", "TCC_EA0_RDREQ_128B"], "wf_req",
                  reader=read_wf_kernels, shard=shard)
    res = {}
    for cls in f:
        if cls not in w or "FETCH_SIZE" not in f[cls] or "WRITE_SIZE" not in w[cls]:
            continue
        rd = 2.0 * f[cls]["FETCH_SIZE"] * 1024.0
        wr = w[cls]["WRITE_SIZE"] * 1024.0
        ns = f[cls]["ns"]
        res[cls] = {"hbm_read_GB": round(rd / 1e9, 3), "hbm_write_GB": round(wr / 1e9, 3), "ms": round(ns / 1e6, 3),
                    "launches": f[cls]["dispatches"],
                    "GBps": round((rd + wr) / max(ns, 1), 1), "frac": round((rd + wr) / max(ns, 1) / HBM_PEAK_GBS, 4)}
        if cls in v:
            res[cls]["valu_counters"] = {k: v[cls][k] for k in v[cls] if k.startswith(("SQ_", "GRBM_"))}
        if cls in ld:
            res[cls]["lds_counters"] = {k: ld[cls][k] for k in ld[cls] if k.startswith(("SQ_", "GRBM_"))}
            res[cls]["lds_counters"]["ns"] = ld[cls]["ns"]
        if cls in rq and "TCC_EA0_RDREQ_128B" in rq[cls]:
            q = rq[cls]
            exact = 32.0 * q.get("TCC_EA0_RDREQ_32B", 0) + 64.0 * q.get("TCC_EA0_RDREQ_64B", 0) + \
                128.0 * q["TCC_EA0_RDREQ_128B"]
            res[cls]["read_requests"] = {"n32": q.get("TCC_EA0_RDREQ_32B"), "n64": q.get("TCC_EA0_RDREQ_64B"),
                                         "n128": q["TCC_EA0_RDREQ_128B"], "all": q.get("TCC_EA0_RDREQ"),
                                         "exact_read_GB": round(exact / 1e9, 3),
                                         "fetch_size_factor": round(exact / (f[cls]["FETCH_SIZE"] * 1024.0), 4)}
    return res


LDS_PEAK_GBS = 150000.0   # MI355X_MICROARCH.md LDS: ~150 TB/s aggregate ds_read_b64/b128, every CU streaming


def lds_block(pmc: dict, cus: int, per_frame: dict) -> dict:
    """The LDS side of the traversal (scene image and stack in LDS): the LDS
    array's busy fraction measured by SQ_LDS_IDX_ACTIVE (all LDS-array cycles,
    summed over CUs) / (CUs x cycles), cycles = GRBM_GUI_ACTIVE / 8 XCDs; and
    the bytes the walk reads from LDS by its own records (16-B sibling pair per
    inner step, 4-B leaf ref, 48-B triangle record per test) over the extend's
    time against the guide's aggregate LDS read rate."""
    if not (pmc.get("SQ_LDS_IDX_ACTIVE") and pmc.get("GRBM_GUI_ACTIVE") and pmc.get("ns")):
        return {}
    cycles = pmc["GRBM_GUI_ACTIVE"] / 8.0
    busy = pmc["SQ_LDS_IDX_ACTIVE"] / (cus * cycles)
    lds_bytes = (16 * per_frame["inner_visits"] + 4 * per_frame["leaf_refs"] + 48 * per_frame["tri_tests"])
    gbs = lds_bytes / pmc["ns"]
    out = {"array_busy_frac": round(busy, 4), "achieved": round(gbs, 1), "peak": LDS_PEAK_GBS, "unit": "GB/s",
           "frac": round(gbs / LDS_PEAK_GBS, 4), "traffic": round(lds_bytes / 1e9, 3),
           "traffic_unit": "GB per frame read from LDS by the walk's records (16 x inner + 4 x leaf refs + 48 x "
                           "triangle tests)",
           "lds_instr_G": round(pmc.get("SQ_INSTS_LDS", 0.0) / 1e9, 3),
           "formula": "array_busy = SQ_LDS_IDX_ACTIVE / (CUs * GRBM_GUI_ACTIVE/8); achieved = traffic / extend ns"}
    if pmc.get("SQ_INSTS_LDS"):
        out["conflict_cycles_per_lds_instr"] = round(pmc.get("SQ_LDS_BANK_CONFLICT", 0.0) / pmc["SQ_INSTS_LDS"], 3)
    return out


def binding_of(roof: dict) -> dict:
    """Which roof the dominant kernel is nearest: the largest of its HBM
    fraction, LDS-array busy fraction and VALU issue fraction."""
    cands = {}
    if roof.get("frac") is not None:
        cands["hbm"] = roof["frac"]
    if roof.get("lds", {}).get("array_busy_frac") is not None:
        cands["lds_array"] = roof["lds"]["array_busy_frac"]
    if roof.get("valu", {}).get("issue_frac") is not None:
        cands["valu_issue"] = roof["valu"]["issue_frac"]
    if not cands:
        return {}
    name = max(cands, key=cands.get)
    return {"binding_frac": cands[name], "binding": name, "fracs": cands}


def valu_block(pmc: dict, cus: int, kern_ms: float, rays: float) -> dict:
    """The resource the traversal is bound by: VALU issue.  A wave64 VALU
    instruction occupies its SIMD for 2 cycles (MI355X_MICROARCH.md), so
    capacity = CUs x 4 SIMDs x cycles / 2; cycles = GRBM_GUI_ACTIVE / 8 XCDs."""
    if not (pmc.get("SQ_INSTS_VALU") and pmc.get("GRBM_GUI_ACTIVE") and kern_ms > 0):
        return {}
    cycles = pmc["GRBM_GUI_ACTIVE"] / 8.0
    issue = pmc["SQ_INSTS_VALU"] / (cus * 4 * cycles / 2.0)
    lanes = (pmc["SQ_THREAD_CYCLES_VALU"] / (64.0 * pmc["SQ_ACTIVE_INST_VALU"])
             if pmc.get("SQ_ACTIVE_INST_VALU") and pmc.get("SQ_THREAD_CYCLES_VALU") else None)
    return {"issue_frac": round(issue, 4),
            "lane_util": round(lanes, 4) if lanes is not None else None,
            "useful_lane_frac": round(issue * lanes, 4) if lanes is not None else None,
            "wave_instr_per_ray": round(pmc["SQ_INSTS_VALU"] / max(rays, 1), 2),
            "clock_GHz_under_pmc": round(cycles / (kern_ms * 1e6), 3),
            "formula": "SQ_INSTS_VALU / (CUs*4*cycles/2); lanes = SQ_THREAD_CYCLES_VALU / (64*SQ_ACTIVE_INST_VALU)"}


def copy_bandwidth(dev, mib: int = 1024, reps: int = 10) -> dict:
    """Stream-copy microbenchmark on this GPU (the measured copy
    bandwidth is the roofline's second denominator): device-to-device copies
    of a 1 GiB buffer, read + write bytes over HIP-event time."""
    import torch
    n = mib * (1 << 20) // 4
    src = torch.ones(n, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    for _ in range(2):
        dst.copy_(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dst.copy_(src)
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1)
    gbs = 2.0 * n * 4 * reps / (ms * 1e-3) / 1e9
    del src, dst
    return {"GBps": round(gbs, 1), "method": f"torch copy_ of {mib} MiB x {reps}, (read + write) bytes / HIP-event time"}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_c1(gpu_rays: int) -> dict:
    """BASELINE.json configs[0] / BASELINE.md section 3: the whole C1 frame
    (Cornell box 512x512, 16 spp, 7 scatters + 1 terminal query) on ONE thread
    of the reference CPU path = the oracle (C restatement of CUTracer.cu:44-218
    with the reference's KD walk, rtx.hlsl:84-211)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test/bench infrastructure only
    from montecarlopathtracer_amd.scenes import scene_path
    oracle.build()
    s = oracle.Scene(scene_path("scene01"))
    p = oracle.RenderParams(width=512, height=512, spp=16, spp_chunk=32, traversal=oracle.KD_REF, threads=1)
    t0 = time.perf_counter()
    _, c = s.render(p)
    dt = time.perf_counter() - t0
    return {"config": "C1 cornell 512x512 16 spp, whole frame, 1 thread", "seconds": round(dt, 3),
            "rays": c["rays"], "paths": c["paths"], "mray_s": round(c["rays"] / dt / 1e6, 4),
            "mpath_s": round(c["paths"] / dt / 1e6, 4), "rays_equal_gpu_c1": c["rays"] == gpu_rays}


def cpu_all_cores(scene_name: str, width: int, height: int, seconds: float, threads: int) -> dict:
    """The same oracle on `threads` host cores over a bounded sample of the GPU
    workload: whole frames (every pixel) at a few samples each, successive
    passes continuing the sample sequence, until `seconds` pass (one thread:
    centred crops, a whole pass would take minutes)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test/bench infrastructure only
    from montecarlopathtracer_amd.scenes import scene_path
    oracle.build()
    s = oracle.Scene(scene_path(scene_name))
    whole = threads > 1
    crop = 64
    spp = 1 if whole else 8
    total_rays, total_paths, total_t = 0, 0, 0.0
    runs = 0
    while total_t < seconds and runs < 1024:
        if whole:
            region = (0, 0, width, height)
        else:
            x0 = (width - crop) // 2 + (runs % 4) * 8
            y0 = (height - crop) // 2 + (runs // 4 % 4) * 8
            region = (x0, y0, x0 + crop, y0 + crop)
        p = oracle.RenderParams(width=width, height=height, spp=spp, spp_chunk=32, spp_offset=runs * spp,
                                traversal=oracle.KD_REF, threads=threads, region=region)
        t0 = time.perf_counter()
        _, c = s.render(p)
        total_t += time.perf_counter() - t0
        total_rays += c["rays"]
        total_paths += c["paths"]
        runs += 1
    what = (f"{runs} whole-frame pass(es) of {spp} spp (samples {0}..{runs * spp - 1})" if whole else
            f"{runs} x ({crop}x{crop} centred crop, {spp} spp)")
    return {"value": round(total_rays / total_t / 1e6, 4), "unit": "Mray/s", "cores": threads,
            "mpath_s": round(total_paths / total_t / 1e6, 4),
            "sample": f"{what} of {scene_name} {width}x{height}, {total_rays} rays in {total_t:.1f}s, "
                      f"{threads} thread(s)"}


def cpu_baseline(scene_name: str, width: int, height: int, seconds: float, threads: int, gpu_c1_rays: int) -> dict:
    c1 = cpu_c1(gpu_c1_rays)
    allc = cpu_all_cores(scene_name, width, height, seconds, threads)
    return {"value": c1["mray_s"], "unit": "Mray/s", "cores": 1, "kind": "port",
            "sample": (f"{c1['config']}: {c1['rays']} rays / {c1['paths']} paths in {c1['seconds']} s "
                       f"({c1['mpath_s']} Mpath/s); oracle = C restatement of CUTracer.cu:44-218 with the "
                       f"reference KD walk rtx.hlsl:84-211; its ray count equals the GPU's C1 render: "
                       f"{c1['rays_equal_gpu_c1']}"),
            "c1": c1, "all_cores": allc, "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            "affinity_cores": host_cores()}


def host_cores() -> int:
    """CPU share of this process (the GPU box gives 16 per GPU; os.cpu_count() shows the host)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", "16"))))


def child_line(args, scene: str, spp: int, steps: int, warmup: int, tag: str, extra: tuple = ()) -> dict:
    """Another BASELINE configuration timed the same way (same pipeline, PMC
    roofline passes) in a child process of this bench (its own GPU context;
    this process's workspace stays allocated beside it)."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--scene", scene, "--no-extra", "--no-alt",
           "--no-cpu-baseline", "--steps", str(steps), "--warmup", str(warmup),
           "--width", str(args.width), "--height", str(args.height), "--spp", str(spp),
           "--spp-chunk", str(args.spp_chunk), "--pipeline", args.pipeline] + (["--no-pmc"] if args.no_pmc else []) + \
        (["--keep-pmc", os.path.join(args.keep_pmc, tag)] if args.keep_pmc else []) + list(extra)
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    except subprocess.TimeoutExpired:
        return {"error": f"{tag} child timed out"}
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"{tag} child rc {r.returncode}: {r.stderr[-400:]}"}
    return json.loads(lines[-1])


def c4_line(args) -> dict:
    """BASELINE configs[3] (C4: the seeded 70k-triangle mesh in scene01's box,
    1024x1024 @ 1024 spp, scene image in global memory with the child-box
    cull), the same steps and warmup as the line."""
    return child_line(args, "cornell_bunny70k", args.spp, args.steps, args.warmup, "c4")


def c5_line(args) -> dict:
    """BASELINE configs[4] (C5: the wavefront pipeline at 4096 spp -- per-bounce
    compaction of live rays into the next queue; the shade runs in queue order,
    the material-sorted shade (wf_sort = 1, the c5_sorted line) renders the
    same image) on ONE GPU: configs[4] names 8 GPUs, which the driver's
    node runs as the main line's N = 8 shares; 3-5 steps (a step is ~1 s)."""
    line = child_line(args, "scene01", 4 * args.spp, max(3, min(args.steps, 5)), 1, "c5")
    if "config" in line:
        line["config"]["shade"] = "queue order (per-bounce compaction by LDS-atomic append); wf_sort=1: same image"
    return line


def c2_sah_line(args) -> dict:
    """The C2 workload on the opt-in SAH KD tree (mcpt_scene_options::kd_build
    = SAH): the same image bit for bit (tests/test_gpu_sah_tree.py), fewer
    node visits.  Not the headline -- the north star keeps the reference's
    KDTree build -- but what a user may switch to.  Same steps, PMC passes."""
    line = child_line(args, "scene01", args.spp, args.steps, args.warmup, "c2_sah", extra=("--kd-build", "sah"))
    return line


def c5_sorted_line(args) -> dict:
    """BASELINE configs[4] as it is worded -- per-bounce compaction PLUS the
    material sort (wf_sort = 1: the shade counting-sorts each block of its queue
    by material in LDS, so a wave runs one material branch) -- on one GPU, 3
    steps, no PMC passes (its extend is the c5 line's; the same image as the
    c5 line, bit for bit)."""
    line = child_line(args, "scene01", 4 * args.spp, 3, 1, "c5_sorted", extra=("--wf-sort", "--no-pmc"))
    if "config" in line:
        line["config"]["shade"] = "material-sorted (wf_sort=1: per-bounce compaction + per-block LDS sort by material)"
    return line


def launch_ranks(args, argv: list) -> int:
    """`--gpus N > 1` started without a launcher (no WORLD_SIZE): run N ranks
    as the driver would -- `torch.distributed.run --nproc-per-node N` on this
    script, as a CHILD process started before this process touches the GPU
    (torch.cuda.device_count() does not initialise it) -- and return its exit
    code; its rank 0 prints the line.  Fewer than N visible GPUs is an error
    (a one-GPU line labelled N GPUs would be unmeasured), except under the
    MCPT_DIST_BACKEND=gloo rehearsal, whose ranks share the GPUs there are."""
    import socket
    import subprocess
    import torch
    n = args.gpus
    have = torch.cuda.device_count()
    if os.environ.get("MCPT_DIST_BACKEND", "nccl") == "nccl" and have < n:
        print(f"bench.py: --gpus {n} but {have} GPU(s) visible; refusing to report a {have}-GPU run as {n}",
              file=sys.stderr, flush=True)
        return 2
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + argv
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def finish_ranks(dist, rank: int, datetime) -> None:
    """Hold ranks 1..N-1 until rank 0 has printed its line, then tear down
    together.  Rank 0's untimed work after the timing (the PMC child processes)
    takes a minute or more; a rank waiting for it inside a collective would hit
    the process group's timeout, and a rank shutting its communicator down
    alone may block in a finalize its peers do not join -- either way the
    launcher ends every rank, rank 0's line included.  The wait is on the
    rendezvous store, which has no watchdog (MCPT_DIST_FINISH_S, default 1200 s),
    and the closing barrier finds every rank present."""
    store = dist.distributed_c10d._get_default_store()
    if rank == 0:
        store.set("mcpt_bench_line_done", "1")
    else:
        store.wait(["mcpt_bench_line_done"],
                   datetime.timedelta(seconds=int(os.environ.get("MCPT_DIST_FINISH_S", "1200"))))
    dist.barrier()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="scene01")
    ap.add_argument("--layout", choices=["auto", "global"], default="auto",
                    help="scene image placement (mcpt_scene_options::layout): LDS when it fits, or global memory "
                         "with child-box records")
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--spp-chunk", type=int, default=32)
    # default: the wavefront pipeline (bit-identical image; C2 13.2 vs 11.7 G rays/s on
    # one MI355X); N = 1 runs also time the megakernel for comparison
    ap.add_argument("--pipeline", choices=["megakernel", "wavefront"], default="wavefront")
    ap.add_argument("--no-alt", action="store_true", help="skip the other pipeline's comparison timing (N = 1)")
    ap.add_argument("--wf-batch", type=int, default=0)
    ap.add_argument("--wf-streams", type=int, default=0, help="wavefront streams (0 = the library's default)")
    ap.add_argument("--kd-build", choices=["reference", "sah"], default="reference",
                    help="KD split rule (mcpt_scene_options::kd_build): the reference's KDTree.hpp rule (the "
                         "headline) or the opt-in SAH with a traversal cost (same image, fewer node visits)")
    ap.add_argument("--no-sah", action="store_true",
                    help="N = 1: skip the C2 line on the SAH tree reported under extra_lines.c2_sah_tree")
    ap.add_argument("--wf-sort", action="store_true",
                    help="wavefront: the material-sorted shade (mcpt_render_params::wf_sort = 1; same image)")
    ap.add_argument("--single-process", action="store_true",
                    help="one process drives all --gpus devices through mcpt_init(devices) (the C ABI's "
                         "multi-device render: replicas, peer-copy gather) instead of one rank per GPU")
    ap.add_argument("--gather", choices=["peer", "rccl"], default="peer",
                    help="--single-process: how the shards reach device 0 (mcpt_render_params::gather): peer "
                         "copies or one ncclGather over a communicator of the device list")
    ap.add_argument("--devices", default="", help="--single-process device list (default 0..gpus-1); a repeated "
                                                  "ordinal rehearses the multi-device path on one GPU, e.g. 0,0")
    ap.add_argument("--set", action="append", default=[], metavar="FIELD=VALUE",
                    help="set a scheduling field of the render params (wf_refill, ready_thresh, wf_group_shift, "
                         "tail_units_per_lane, wf_mem_limit, ...; never changes the image) -- for sweeps")
    ap.add_argument("--keep-pmc", default="", help="copy the raw rocprofv3 PMC csv files into this directory")
    ap.add_argument("--dump-image", default="", help="rank 0 saves the last timed step's (gathered) image here "
                                                     "as a (H, W, 4) float32 .npy (tests)")
    ap.add_argument("--pmc-shard", default="1,0", help=argparse.SUPPRESS)   # PMC child: shard count,index
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = this process's CPU share (<= 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c4", action="store_true",
                    help="N = 1: skip the C4 line (BASELINE configs[3], the 70k-triangle mesh in the Cornell box, "
                         "same pipeline, steps and PMC roofline) reported under extra_lines.c4")
    ap.add_argument("--no-c5", action="store_true",
                    help="N = 1: skip the C5 line (BASELINE configs[4], the wavefront at 4096 spp on one GPU, "
                         "3-5 steps, PMC roofline) reported under extra_lines.c5")
    ap.add_argument("--no-extra", action="store_true", help="skip both extra lines (--no-c4 --no-c5)")
    ap.add_argument("--counting", action="store_true", help="time the counting megakernel instead of the lean one")
    ap.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 PMC passes (HBM bytes, VALU issue)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)   # one render under rocprofv3
    args = ap.parse_args()
    if args.no_extra:
        args.no_c4 = args.no_c5 = args.no_sah = True
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.single_process and not args.pmc_child:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if not args.pmc_child and not args.single_process and world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched")

    import datetime
    import torch
    import torch.distributed as dist
    import montecarlopathtracer_amd as M

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MCPT_DIST_BACKEND=gloo: rehearsal of the N > 1 path with every rank on the
    # GPUs this box has (local % device_count) and the gather staged through host
    # memory; the driver's multi-GPU runs use the default, RCCL ("nccl").
    backend = os.environ.get("MCPT_DIST_BACKEND", "nccl")
    if world > 1 and args.single_process:
        raise SystemExit("--single-process drives every GPU from one process: launch it without torch.distributed.run")
    if world > 1:
        if backend == "nccl" and local >= torch.cuda.device_count():
            raise SystemExit(f"bench.py: rank {rank} (local {local}) has no GPU: "
                             f"{torch.cuda.device_count()} visible for {world} ranks")
        local = local % max(torch.cuda.device_count(), 1) if backend == "gloo" else local
        torch.cuda.set_device(local)
        # bounded: a stuck RCCL set-up exits non-zero inside the driver's limit
        tmo = datetime.timedelta(seconds=int(os.environ.get("MCPT_DIST_TIMEOUT_S", "180")))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
    dev = torch.device("cuda", local if world > 1 else 0)
    red_dev = dev if backend == "nccl" else torch.device("cpu")   # device of the small timing reductions
    torch.cuda.set_device(dev)
    # --single-process: one process, the C ABI's device list (mcpt_init): scenes are
    # replicated on every device and each render is split into interleaved-tile
    # shards gathered to device 0 by peer copies (capi.cpp render_multi)
    n_dev = args.gpus if args.single_process else 1
    devices = [int(x) for x in args.devices.split(",")] if args.devices else list(range(n_dev))
    if args.single_process and (len(devices) != n_dev or max(devices) >= torch.cuda.device_count()):
        raise SystemExit(f"--single-process --gpus {n_dev}: device list {devices}, "
                         f"{torch.cuda.device_count()} device(s) visible")
    M.Tracer().initialize(devices if n_dev > 1 else [dev.index])
    n_gpus = world * n_dev
    if not args.pmc_child and n_gpus != args.gpus:    # never a line whose n_gpus is not --gpus
        raise SystemExit(f"bench.py: --gpus {args.gpus} but {n_gpus} GPU(s) would render")

    scene = M.Scene(M.ObjModel(M.scene_path(args.scene)), layout=args.layout, kd_build=args.kd_build)
    scene_id = 2 if args.scene in ("scene02", "scene03") else 1
    if args.pmc_child:   # PMC pass: exactly one render of the timed kernel (rank 0's shard), then exit
        sc, si = (int(x) for x in args.pmc_shard.split(","))
        p = M.RenderParams.for_scene(scene_id, width=args.width, height=args.height, spp=args.spp,
                                     spp_chunk=args.spp_chunk, tile=8, pipeline=args.pipeline, wf_batch=args.wf_batch,
                                     wf_streams=args.wf_streams, shard_count=sc, shard_index=si, packed=sc > 1,
                                     lean=not args.counting, wf_sort=args.wf_sort, **_tuning(args))
        fb = torch.zeros((p.output_pixels(), 4), dtype=torch.float32, device=dev)
        scene.render_device(p, fb.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        return
    # timed renders run the lean kernels (no per-step traversal counters, same
    # image and ray count); the node/leaf/triangle counts of the bytes model come
    # from one untimed counting render of the same frame (they are deterministic)
    lean = not args.counting
    p = M.RenderParams.for_scene(scene_id, width=args.width, height=args.height, spp=args.spp,
                                 spp_chunk=args.spp_chunk, tile=8, shard_count=world, shard_index=rank,
                                 packed=world > 1, pipeline=args.pipeline, wf_batch=args.wf_batch,
                                 wf_streams=args.wf_streams, lean=lean, gather=args.gather, wf_sort=args.wf_sort,
                                 **_tuning(args))
    p_count = dataclasses.replace(p, lean=False)
    n_out = p.output_pixels()
    fb = torch.zeros((n_out, 4), dtype=torch.float32, device=dev)
    scene.reserve(p)
    plan = scene.plan(p)
    stream = torch.cuda.current_stream(dev)

    gatherer = None
    if world > 1:
        from montecarlopathtracer_amd.sharding import TileGather
        gatherer = TileGather(args.width, args.height, world, rank, dev, tile=8)

    def step():
        scene.render_device(p, fb.data_ptr(), stream.cuda_stream)
        if gatherer is not None:
            gatherer.gather(fb)   # RCCL gather of the packed tile buffers + unpermute on rank 0

    scene.stats()
    scene.render_device(p_count, fb.data_ptr(), stream.cuda_stream)   # untimed counting render
    torch.cuda.synchronize(dev)
    counts = scene.stats()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    scene.stats()   # reset counters/timers after warmup

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    for d in sorted(set(devices)) if n_dev > 1 else [dev]:
        torch.cuda.synchronize(d)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = scene.stats()   # waits for the recorded HIP events of each path-kernel launch

    # the other pipeline on the same frame, for comparison (N = 1; same image, bit for bit)
    alt = None
    if args.dump_image and rank == 0:   # before the comparison renders reuse fb
        import numpy as np
        img = gatherer.image if gatherer is not None else fb
        np.save(args.dump_image, img.view(args.height, args.width, 4).cpu().numpy())
    if n_gpus == 1 and not args.no_alt:
        other = "megakernel" if args.pipeline == "wavefront" else "wavefront"
        pa = dataclasses.replace(p, pipeline=other)
        for _ in range(max(args.warmup, 1)):
            scene.render_device(pa, fb.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
        scene.stats()
        ta = time.perf_counter()
        for _ in range(args.steps):
            scene.render_device(pa, fb.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
        ta = time.perf_counter() - ta
        sa = scene.stats()
        alt = {"pipeline": other, "value": round(sa["rays"] / ta / 1e6, 3), "unit": "Mray/s",
               "ms_per_step": round(ta / args.steps * 1e3, 3),
               "kernel_ms_avg": round(sa["kernel_ms"] / max(sa["renders"], 1), 3),
               "rays_equal": sa["rays"] == st["rays"]}

    # per-render node/leaf/triangle counts: the counting render's (identical for a lean one)
    renders = max(st["renders"], 1)
    for k in ("paths", "inner_visits", "leaf_visits", "leaf_refs", "tri_tests", "shades", "stack_spills"):
        if lean:
            st[k] = counts[k] * renders
    counts_match = counts["rays"] * renders == st["rays"]
    count_keys = ("rays", "paths", "inner_visits", "leaf_visits", "leaf_refs", "tri_tests", "shades", "stack_spills")
    kern_ms = st["kernel_ms"] / renders
    if world > 1:
        # whole-job counts (every rank's shard) and the slowest rank's time
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0].item()), float(t[1].item())
        agg = torch.tensor([st[k] for k in count_keys], dtype=torch.float64, device=red_dev)
        dist.all_reduce(agg, op=dist.ReduceOp.SUM)
        for i, k in enumerate(count_keys):
            st[k] = int(agg[i].item())
    rays = st["rays"]

    if rank == 0:
        per_launch = {k: st[k] / renders for k in count_keys}
        ab = algorithmic_bytes(per_launch, args.width * args.height)
        algo_gbs = ab["survey"] / (kern_ms * 1e-3) / 1e9
        mray = rays / elapsed / 1e6
        workload = f"cornell_{args.width}x{args.height}_{args.spp}spp" + ("" if args.scene == "scene01" else
                                                                            f"_{args.scene}") + \
            ("" if args.kd_build == "reference" else f"_kd_{args.kd_build}")
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        # the PMC passes profile one device's share: rank 0's shard (N > 1) or the whole frame
        shard = (n_gpus, 0) if n_gpus > 1 else (1, 0)
        roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                "traffic": None, "traffic_unit": None,
                "source": "rocprofv3 --pmc passes of this build and workload, run by this bench"
                          + (f" on rank 0's shard ({shard[1]} of {shard[0]})" if n_gpus > 1 else "")}
        if not args.no_pmc and args.pipeline == "wavefront":
            # the dominant kernel is wf_extend (the traversal): `achieved` = its measured HBM bytes
            # (FETCH_SIZE x2 + WRITE_SIZE of its dispatches over one frame) / the same dispatches'
            # duration in the PMC pass, which serializes the kernels; the whole pipeline's queue
            # traffic over the frame's HIP-event time is reported separately under `pipeline`
            kh = wavefront_hbm(args, shard)
            ext = kh.get("extend")
            if ext:
                eb = ext["hbm_read_GB"] + ext["hbm_write_GB"]
                gbs = eb / (ext["ms"] * 1e-3) if ext["ms"] > 0 else 0.0
                roof.update(achieved=round(gbs, 2), frac=round(gbs / HBM_PEAK_GBS, 5), traffic=round(eb, 3),
                            traffic_unit="GB of HBM read+write per frame by wf_extend's dispatches",
                            kernel="wf_extend (the traversal, the dominant kernel)",
                            launches=ext["launches"], kernel_ms=ext["ms"],
                            avg_launch_ms=round(ext["ms"] / max(ext["launches"], 1), 4),
                            timing="sum of the extend dispatches' durations in the PMC pass (kernels serialized)")
                rr = ext.get("read_requests")
                if rr:
                    # the extend's ray stream (ray_stream_bytes) against the exact fabric reads: the rest
                    # is node / triangle records (and stack refills) fetched past the L2
                    shard_rays, shard_paths = per_launch["rays"] / n_gpus, per_launch["paths"] / n_gpus
                    ray_gb = ray_stream_bytes(shard_rays, shard_paths, st["variant"]) / 1e9
                    roof["read_split"] = {
                        "exact_read_GB": rr["exact_read_GB"], "fetch_size_factor": rr["fetch_size_factor"],
                        "ray_GB": round(ray_gb, 3), "record_GB": round(rr["exact_read_GB"] - ray_gb, 3),
                        "hit_id_write_GB": round(hit_write_bytes(shard_rays) / 1e9, 3),
                        "spill_write_GB": round(16.0 * per_launch["stack_spills"] / n_gpus / 1e9, 3),
                        "method": "TCC_EA0_RDREQ_{32B,64B,128B} pass: exact = 32 n32 + 64 n64 + 128 n128 (every "
                                  "request 128 B here; FETCH_SIZE counts 64 B each, factor 2 exactly, "
                                  "scripts/fetch_calib.hip); ray_GB from the counted rays / paths "
                                  "(bench.ray_stream_bytes)"}
                vb = valu_block(ext.pop("valu_counters", {}), cus, ext.get("ms", 0.0), per_launch["rays"] / n_gpus)
                if vb:
                    vb["kernel"] = "wf_extend (the traversal: the dominant kernel), run alone"
                    roof["valu"] = vb
                # rank 0's shard: its share of the frame's counts (interleaved tiles, ~1/N)
                lb = lds_block(ext.pop("lds_counters", {}), cus,
                               {k: per_launch[k] / n_gpus for k in ("inner_visits", "leaf_refs", "tri_tests")})
                if lb and st["variant"] == 4:    # scene image in LDS (the global variant's LDS holds only stacks)
                    lb["kernel"] = "wf_extend, run alone"
                    roof["lds"] = lb
                roof.update(binding_of(roof))
            for k in kh.values():
                k.pop("valu_counters", None)
                k.pop("lds_counters", None)
            if kh:
                tot_b = sum((k["hbm_read_GB"] + k["hbm_write_GB"]) for k in kh.values())
                pg = tot_b / (kern_ms * 1e-3) if kern_ms > 0 else 0.0
                roof["pipeline"] = {
                    "achieved": round(pg, 2), "frac": round(pg / HBM_PEAK_GBS, 5), "unit": "GB/s",
                    "traffic": round(tot_b, 3), "traffic_unit": "GB of HBM per frame, all wavefront kernels "
                                                                "(mostly the SoA queue streams)",
                    "frame_ms": round(kern_ms, 3), "kernels": kh,
                    "note": "per-kernel ms / GBps from the PMC passes, which run kernels one at a time; the timed "
                            "frame overlaps them on several streams (frame_ms = HIP events of the timed renders)"}
        elif not args.no_pmc:
            # measured HBM bytes: FETCH_SIZE x2 (gfx950 streaming-read undercount) + WRITE_SIZE, KiB
            pmc = live_counters(args)
            if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
                hbm = (2.0 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024.0
                gbs = hbm / (kern_ms * 1e-3) / 1e9
                roof.update(achieved=round(gbs, 2), frac=round(gbs / HBM_PEAK_GBS, 5), traffic=round(hbm / 1e9, 3),
                            traffic_unit="GB of HBM read+write per path-kernel launch", kernel="path_kernel",
                            hbm_read_GB=round(2.0 * pmc["FETCH_SIZE"] * 1024 / 1e9, 3),
                            hbm_write_GB=round(pmc["WRITE_SIZE"] * 1024 / 1e9, 3))
            vb = valu_block(pmc, cus, kern_ms, per_launch["rays"] / n_gpus)
            if vb:
                roof["valu"] = vb
        cb = copy_bandwidth(dev)
        if roof["achieved"] is not None and cb["GBps"] > 0:
            cb["achieved_frac"] = round(roof["achieved"] / cb["GBps"], 5)
        roof["peak_copy_measured"] = cb
        for k in roof.get("pipeline", {}).get("kernels", {}).values():
            k["frac_of_copy"] = round(k["GBps"] / cb["GBps"], 4) if cb["GBps"] > 0 else None
        in_lds = st["variant"] in (1, 2, 4)   # kernel variants that hold the scene image in LDS
        if not in_lds:
            roof["binding_resource"] = ("memory latency of the node / triangle reads (scene image in global memory, "
                                        "served by L1/L2/MALL; profiles/r02/c4_mem)")
        elif args.pipeline == "wavefront":
            roof["binding_resource"] = ("wf_extend: VALU issue x lane use (valu.useful_lane_frac; scene image in "
                                        "LDS, so its HBM bytes are ray reads and hit writes only); the queue "
                                        "streams that generate / shade / accumulate move beside it are under "
                                        "pipeline")
        else:
            roof["binding_resource"] = ("VALU issue and lane divergence (the scene image is LDS-resident; HBM "
                                        "carries only stack spills and the framebuffer partials)")
        roof["algorithmic"] = {"GBps": round(algo_gbs, 1), "bytes_per_ray": round(ab["survey"] / max(per_launch["rays"], 1), 1),
                               "bytes_per_launch": int(ab["survey"]),
                               "model": "SURVEY 8(d): 32*nodes+4*leafrefs+48*tris+96*shades+16*px",
                               "served_from": ("LDS (scene image) and L2 (normals), not HBM" if in_lds else
                                               "L1 / L2 / MALL (scene image in global memory)"),
                               "own_layout_GBps": round(ab["own"] / (kern_ms * 1e-3) / 1e9, 1),
                               "per_ray": {k: round(per_launch[k] / max(per_launch["rays"], 1), 3) for k in
                                           ("inner_visits", "leaf_visits", "leaf_refs", "tri_tests", "shades")}}
        sched = {k: plan[k] for k in ("wf_streams", "wf_batch", "wf_batch_default", "wf_refill", "wf_group_shift")
                 if args.pipeline == "wavefront"} if args.pipeline == "wavefront" else \
            {k: plan[k] for k in ("ready_thresh", "tail_units")}
        sched["workspace_GB"] = round(plan["workspace_bytes"] / 1e9, 2)
        if n_gpus > 1:
            par = (f"pixel-tiles x{n_gpus} + " + (f"{'rccl' if backend == 'nccl' else backend} gather" if world > 1
                                                  else f"{'peer-copy' if args.gather == 'peer' else 'rccl'} gather "
                                                       f"(one process, mcpt_init({devices}))"))
        else:
            par = "pixel-tiles x1"
        line = {
            "metric": METRIC, "value": round(mray, 3), "unit": "Mray/s", "n_gpus": n_gpus, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": f"bundled reference scene {args.scene}.obj (Cornell Box), synthetic camera/seed",
            "config": {"workload": workload, "scene": args.scene,
                       "width": args.width, "height": args.height, "spp": args.spp, "max_depth": 7,
                       "spp_chunk": args.spp_chunk, "parallelism": par, "pipeline": args.pipeline,
                       "wf_sort": bool(args.wf_sort), "kd_build": args.kd_build,
                       "kd_nodes": scene.info()["n_nodes"],
                       "kernel_variant": st["variant"], "schedule": sched},
            "rays_per_step": rays // args.steps,
            "paths_per_step": st["paths"] // args.steps,
            "mpath_s": round(st["paths"] / elapsed / 1e6, 3),
            "rays_per_path": round(st["rays"] / max(st["paths"], 1), 4),
            "stack_spills_per_ray": round(st["stack_spills"] / max(st["rays"], 1), 4),
            "timed_kernel": (f"lean {'megakernel' if args.pipeline == 'megakernel' else 'wavefront extend'} "
                             "(traversal counters compiled out)") if lean else "counting",
            "counts_source": ("untimed counting render of the same frame; its rays equal the timed "
                              f"renders': {counts_match}") if lean else "timed renders",
            "kernel_ms_avg": round(kern_ms, 3),
            "gpu_ms_per_step_event": round(ev0.elapsed_time(ev1) / args.steps, 3),
            "roofline": roof,
            "cpu_baseline": None,
            "other_pipeline": alt,
        }
        if n_gpus == 1 and args.scene == "scene01":
            extra = {}
            if not args.no_c4:
                extra["c4"] = c4_line(args)
            if not args.no_sah and args.kd_build == "reference":
                extra["c2_sah_tree"] = c2_sah_line(args)
            if not args.no_c5 and args.spp == 1024 and args.pipeline == "wavefront":
                extra["c5"] = c5_line(args)
                extra["c5_sorted"] = c5_sorted_line(args)
            if extra:
                line["extra_lines"] = extra
        if n_gpus == 1 and not args.no_cpu_baseline:
            # the GPU's own C1 frame, for the ray-count check of the CPU run
            s1 = scene if args.scene == "scene01" else M.Scene(M.ObjModel(M.scene_path("scene01")))
            _, c1 = s1.render(M.RenderParams(width=512, height=512, spp=16, spp_chunk=32))
            line["cpu_baseline"] = cpu_baseline(args.scene, args.width, args.height, args.cpu_seconds,
                                                args.cpu_threads or host_cores(), c1["rays"])
        print(json.dumps(line), flush=True)
    if world > 1:
        finish_ranks(dist, rank, datetime)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
