"""Time one rank's share of C2 (1024^2 x 1024 spp, shard r of N) on this GPU,
megakernel vs wavefront at several batch sizes (what an N-GPU run's rank sees)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import montecarlopathtracer_amd as M  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
scene = M.Scene(M.ObjModel(M.scene_path("scene01")))
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
for pipe, batch in (("megakernel", 0), ("wavefront", 0), ("wavefront", 1 << 26), ("wavefront", 1 << 25)):
    p = M.RenderParams(width=1024, height=1024, spp=1024, spp_chunk=32, tile=8, shard_count=N, shard_index=0,
                       packed=True, pipeline=pipe, wf_batch=batch, lean=True)
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
    print(f"N={N} {pipe} batch={batch}: {dt * 1e3:.1f} ms, {st['rays'] / 3 / dt / 1e9:.2f} G rays/s", flush=True)
    del fb
