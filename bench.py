#!/usr/bin/env python3
"""bench.py -- Cornell Box 1024x1024 @ 1024 spp on N MI355X (BASELINE.json configs[1]/[2]).

One step = one full path-traced frame of the workload (every pixel, every
sample, up to 7 scatter events + 1 terminal query per path) through the C ABI
(mcpt_render_device), plus -- for N > 1 -- the RCCL gather of the per-rank
tile buffers to rank 0 and its unpermute into the image.  Pixels are sharded
as interleaved 8x8 tiles (tile t -> rank t % N); total work is fixed, so the
scaling is strong.  value = closest-hit queries of all ranks / max-over-ranks
wall time (Mray/s).

Launch:  python bench.py [--gpus 1 --steps 3 --warmup 1]
         python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
             --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...
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


def pmc_traffic(workload: str, pipeline: str):
    """HBM bytes per path-kernel launch (GB) from the committed rocprofv3 PMC passes
    (profiles/<round>/pmc_summary.json: FETCH_SIZE x2 gfx950 correction + WRITE_SIZE,
    scripts/profile_round.sh) when they were taken on this workload; else None."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_summary.json")), reverse=True):
        try:
            d = json.load(open(f))
            bl = d.get("bench_line") or {}
            if bl.get("config", {}).get("workload") == workload and \
                    bl.get("config", {}).get("pipeline", "megakernel") == pipeline:
                g = d["derived"]
                return round(g["hbm_read_GB_corrected_x2"] + g["hbm_write_GB"], 3), os.path.relpath(f, ROOT)
        except (OSError, ValueError, KeyError):
            continue
    return None, None


def cpu_baseline(scene_name: str, width: int, height: int, seconds: float, threads: int) -> dict:
    """Reference CPU path = the oracle (C restatement of CUTracer.cu + the reference
    KD traversal rtx.hlsl:84-211, pthreads over rows) on `threads` host cores, on a
    bounded sample of the workload: centred crops rendered until `seconds` pass."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test/bench infrastructure only
    from montecarlopathtracer_amd.scenes import scene_path
    oracle.build()
    s = oracle.Scene(scene_path(scene_name))
    crop = 64 if threads == 1 else 256
    spp = 8
    total_rays, total_t = 0, 0.0
    runs = 0
    while total_t < seconds and runs < 1024:
        x0 = (width - crop) // 2 + (runs % 4) * 8
        y0 = (height - crop) // 2 + (runs // 4 % 4) * 8
        p = oracle.RenderParams(width=width, height=height, spp=spp, spp_chunk=32, spp_offset=runs * spp,
                                traversal=oracle.KD_REF, threads=threads, region=(x0, y0, x0 + crop, y0 + crop))
        t0 = time.perf_counter()
        _, c = s.render(p)
        total_t += time.perf_counter() - t0
        total_rays += c["rays"]
        runs += 1
    return {"value": round(total_rays / total_t / 1e6, 4), "unit": "Mray/s", "cores": threads, "kind": "port",
            "sample": f"{runs} x ({crop}x{crop} centred crop, {spp} spp) of {scene_name} {width}x{height}, "
                      f"{total_rays} rays in {total_t:.1f}s, oracle traversal=KD_REF (rtx.hlsl order), "
                      f"{threads} thread(s)"}


def host_cores() -> int:
    """CPU share of this process (the GPU box gives 16 per GPU; os.cpu_count() shows the host)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", "16"))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="scene01")
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--spp-chunk", type=int, default=32)
    ap.add_argument("--pipeline", choices=["megakernel", "wavefront"], default="megakernel")
    ap.add_argument("--wf-batch", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = this process's CPU share (<= 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--counting", action="store_true", help="time the counting megakernel instead of the lean one")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import montecarlopathtracer_amd as M

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MCPT_DIST_BACKEND=gloo: rehearsal of the N > 1 path with every rank on the
    # GPUs this box has (local % device_count) and the gather staged through host
    # memory; the driver's multi-GPU runs use the default, RCCL ("nccl").
    backend = os.environ.get("MCPT_DIST_BACKEND", "nccl")
    if world > 1:
        local = local % max(torch.cuda.device_count(), 1) if backend == "gloo" else local
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local if world > 1 else 0)
    red_dev = dev if backend == "nccl" else torch.device("cpu")   # device of the small timing reductions
    torch.cuda.set_device(dev)
    M.Tracer().initialize([dev.index])

    scene = M.Scene(M.ObjModel(M.scene_path(args.scene)))
    scene_id = 2 if args.scene in ("scene02", "scene03") else 1
    # timed renders run the megakernel lean (no per-step traversal counters, same
    # image and ray count); the node/leaf/triangle counts of the bytes model come
    # from one untimed counting render of the same frame (they are deterministic)
    lean = args.pipeline == "megakernel" and not args.counting
    p = M.RenderParams.for_scene(scene_id, width=args.width, height=args.height, spp=args.spp,
                                 spp_chunk=args.spp_chunk, tile=8, shard_count=world, shard_index=rank,
                                 packed=world > 1, pipeline=args.pipeline, wf_batch=args.wf_batch, lean=lean)
    p_count = dataclasses.replace(p, lean=False)
    n_out = p.output_pixels()
    fb = torch.zeros((n_out, 4), dtype=torch.float32, device=dev)
    scene.reserve(p)
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
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = scene.stats()   # waits for the recorded HIP events of each path-kernel launch

    rays = st["rays"]
    # per-render node/leaf/triangle counts: the counting render's (identical for a lean one)
    renders = max(st["renders"], 1)
    for k in ("paths", "inner_visits", "leaf_visits", "leaf_refs", "tri_tests", "shades", "stack_spills"):
        if lean:
            st[k] = counts[k] * renders
    counts_match = counts["rays"] * renders == st["rays"]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        agg = torch.tensor([st[k] for k in ("rays", "paths", "inner_visits", "leaf_visits", "leaf_refs",
                                              "tri_tests", "shades")] + [st["kernel_ms"]],
                           dtype=torch.float64, device=red_dev)
        dist.all_reduce(agg, op=dist.ReduceOp.SUM)
        rays = int(agg[0].item())

    if rank == 0:
        per_launch = {k: st[k] / max(st["renders"], 1) for k in
                      ("rays", "inner_visits", "leaf_visits", "leaf_refs", "tri_tests", "shades")}
        kern_ms = st["kernel_ms"] / max(st["renders"], 1)
        ab = algorithmic_bytes(per_launch, n_out)
        achieved = ab["survey"] / (kern_ms * 1e-3) / 1e9
        achieved_own = ab["own"] / (kern_ms * 1e-3) / 1e9
        mray = rays / elapsed / 1e6
        workload = f"cornell_{args.width}x{args.height}_{args.spp}spp" + ("" if args.scene == "scene01" else
                                                                            f"_{args.scene}")
        # the committed PMC passes are single-GPU launches of the whole frame
        traffic, traffic_src = pmc_traffic(workload, args.pipeline) if world == 1 else (None, None)
        line = {
            "metric": METRIC, "value": round(mray, 3), "unit": "Mray/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": f"bundled reference scene {args.scene}.obj (Cornell Box), synthetic camera/seed",
            "config": {"workload": workload, "scene": args.scene,
                       "width": args.width, "height": args.height, "spp": args.spp, "max_depth": 7,
                       "spp_chunk": args.spp_chunk, "parallelism": f"pixel-tiles x{world}" +
                       (f" + {'rccl' if backend == 'nccl' else backend} gather" if world > 1 else ""), "pipeline": args.pipeline,
                       "kernel_variant": st["variant"]},
            "rays_per_step": rays // args.steps,
            "rays_per_path": round(st["rays"] / max(st["paths"], 1), 4),
            "stack_spills_per_ray": round(st["stack_spills"] / max(st["rays"], 1), 4),
            "timed_kernel": "lean megakernel (traversal counters compiled out)" if lean else "counting",
            "counts_source": ("untimed counting render of the same frame; its rays equal the timed "
                              f"renders': {counts_match}") if lean else "timed renders",
            "kernel_ms_avg": round(kern_ms, 3),
            "gpu_ms_per_step_event": round(ev0.elapsed_time(ev1) / args.steps, 3),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_unit": "GB per launch (HBM read+write, rocprofv3 PMC)", "traffic_source": traffic_src,
                         "bytes_model": "SURVEY 8(d): 32*nodes+4*leafrefs+48*tris+96*shades+16*px",
                         "note": ("frac > 1: the algorithmic bytes are served from LDS (scene image) and L2 "
                                  "(normals), not HBM -- see traffic; the kernel is bound by VALU issue and "
                                  "lane divergence (DESIGN.md section 5)"),
                         "achieved_own_layout": round(achieved_own, 1),
                         "bytes_per_ray": round(ab["survey"] / max(per_launch["rays"], 1), 1),
                         "per_ray": {k: round(per_launch[k] / max(per_launch["rays"], 1), 3) for k in
                                     ("inner_visits", "leaf_visits", "leaf_refs", "tri_tests", "shades")}},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.scene, args.width, args.height, args.cpu_seconds,
                                                args.cpu_threads or host_cores())
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
