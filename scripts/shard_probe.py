"""Time one rank's share of C2 (1024^2 x 1024 spp, shard 0 of N) on this GPU
-- what an N-GPU run's rank renders -- for the megakernel and wavefront
schedules (streams x batch).  usage: shard_probe.py N [N ...] [--combos s:b,s:b,...]
(b = paths per batch, 0 = automatic; s = streams, 0 = automatic)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import montecarlopathtracer_amd as M  # noqa: E402

args = sys.argv[1:]
combos = [(0, 0), (3, 0), (4, 0)]
if "--combos" in args:
    i = args.index("--combos")
    combos = [tuple(int(v) for v in c.split(":")) for c in args[i + 1].split(",")]
    args = args[:i] + args[i + 2:]
NS = [int(x) for x in args] or [8]
scene = M.Scene(M.ObjModel(M.scene_path("scene01")))
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
runs = [(n, "megakernel", 0, 0) for n in NS] + [(n, "wavefront", s, b) for n in NS for s, b in combos]
for N, pipe, streams, batch in runs:
    p = M.RenderParams(width=1024, height=1024, spp=1024, spp_chunk=32, tile=8, shard_count=N, shard_index=0,
                       packed=N > 1, pipeline=pipe, wf_batch=batch, wf_streams=streams, lean=True)
    fb = torch.zeros((p.output_pixels(), 4), dtype=torch.float32, device=dev)
    scene.render_device(p, fb.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    scene.stats()
    t0 = time.perf_counter()
    for _ in range(3):
        scene.render_device(p, fb.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    st = scene.stats()
    plan = scene.plan(p)
    print(f"N={N} {pipe} streams={plan['wf_streams']} batch={plan['wf_batch']}: {dt * 1e3:.1f} ms, "
          f"{st['rays'] / 3 / dt / 1e9:.2f} G rays/s", flush=True)
    del fb
