"""Strong-scaling tail on one GPU: render rank 0's share of an N-way tile split
(what each rank of `bench.py --gpus N` runs) and compare its kernel time with
1/N of the whole frame.  Usage: python scripts/shard_tail.py [--pipeline ...]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import montecarlopathtracer_amd as M  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pipeline", default="megakernel")
ap.add_argument("--spp", type=int, default=1024)
ap.add_argument("--spp-chunk", type=int, default=32)
ap.add_argument("--scene", default="scene01")
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()
dev = torch.device("cuda", 0)
M.Tracer().initialize([0])
scene = M.Scene(M.ObjModel(M.scene_path(args.scene)))
stream = torch.cuda.current_stream(dev)
base = None
for n in (1, 2, 4, 8):
    ms = []
    for rank in ((0, n - 1) if n > 1 else (0,)):
        p = M.RenderParams.for_scene(1, width=1024, height=1024, spp=args.spp, spp_chunk=args.spp_chunk, tile=8,
                                     shard_count=n, shard_index=rank, packed=n > 1, pipeline=args.pipeline)
        fb = torch.zeros((p.output_pixels(), 4), dtype=torch.float32, device=dev)
        scene.reserve(p)
        scene.render_device(p, fb.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
        scene.stats()
        for _ in range(args.reps):
            scene.render_device(p, fb.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
        st = scene.stats()
        ms.append(st["kernel_ms"] / st["renders"])
    t = max(ms)
    base = base or t
    print(json.dumps({"n": n, "pipeline": args.pipeline, "kernel_ms_rank0_last": [round(x, 2) for x in ms],
                      "ideal_ms": round(base / n, 2), "efficiency": round(base / (n * t), 4)}), flush=True)
