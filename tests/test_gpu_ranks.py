"""The N > 1 paths on the GPU, as the driver's multi-GPU runs will first execute
them (BASELINE configs[2]: pixel tiles across ranks + a tile gather to rank 0).

* bench.py's rank path with world_size 2 and 8 (torch.distributed.run, gloo,
  every rank on GPU 0): rank 0's gathered image equals the single-GPU render bit
  for bit, and the JSON line carries n_gpus == 2 and the roofline of rank 0's
  shard.  RCCL itself needs two distinct GPUs (a communicator refuses a
  repeated device), so the driver's 8-GPU node is where "nccl" first runs;
  everything around the collective -- the shard params, the packed wavefront
  renders, TileGather's slot map and unpermute, the max-over-ranks timing --
  is what runs here.
* the same over torch.multiprocessing (spawned before any GPU call of theirs):
  each rank renders its tiles on the GPU and TileGather reassembles them --
  test_sharding_gloo.py's CPU test with GPU renders instead of oracle slices.
* one process, the C ABI's device list (bench.py --single-process --devices
  0,0): the same image.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, SPP = 256, 192, 16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _single_gpu_image(mcpt, pipeline="wavefront", w=W, h=H):
    scene = mcpt.Scene(mcpt.ObjModel(mcpt.scene_path("scene01")))
    img, st = scene.render(mcpt.RenderParams(width=w, height=h, spp=SPP, spp_chunk=32, pipeline=pipeline))
    return img, st


def _bench_line(stdout: str) -> dict:
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


# world 8: the driver's N = 8 dealing with an uneven tile split (33 x 25 tiles
# of 8 x 8 = 825 over 8 ranks: 104 for rank 0, 103 for the others, so
# TileGather pads to the largest shard), all eight ranks on GPU 0; rank 0's
# PMC passes only at world 2 (the roofline plumbing), not repeated at 8
@pytest.mark.parametrize("world,w,h,pmc", [(2, W, H, True), (8, 264, 200, False)])
def test_bench_rank_path_gloo(mcpt, tmp_path, world, w, h, pmc):
    out = str(tmp_path / "img.npy")
    env = dict(os.environ, MCPT_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--width", str(w), "--height", str(h),
           "--spp", str(SPP), "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--dump-image", out]
    if not pmc:
        cmd.append("--no-pmc")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = _bench_line(r.stdout)
    assert line["n_gpus"] == world and line["value"] > 0
    assert "gloo gather" in line["config"]["parallelism"]
    roof = line["roofline"]
    assert roof["bound"] == "hbm" and roof["peak"] > 0 and "source" in roof
    if pmc and roof["achieved"] is not None:      # rocprofv3 present: rank 0's shard measured
        assert roof["frac"] > 0 and "rank 0's shard" in roof["source"]
    got = np.load(out)
    ref, st = _single_gpu_image(mcpt, w=w, h=h)
    assert np.array_equal(got[..., :3], ref)
    # whole-job rays: both ranks' shards = the single-GPU frame's rays per step
    assert line["rays_per_step"] == st["rays"]


def _worker(rank, world, port, pipeline, out_path):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    import montecarlopathtracer_amd as M
    from montecarlopathtracer_amd.sharding import TileGather, shard_params
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    scene = M.Scene(M.ObjModel(M.scene_path("scene01")))
    p = shard_params(M.RenderParams(width=W, height=H, spp=SPP, spp_chunk=32, pipeline=pipeline), world, rank)
    fb = torch.zeros((p.output_pixels(), 4), dtype=torch.float32, device=dev)
    scene.render_device(p, fb.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    g = TileGather(W, H, world, rank, dev)
    out = g.gather(fb)
    if rank == 0:
        np.save(out_path, out.view(H, W, 4).cpu().numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("pipeline", ["wavefront", "megakernel"])
def test_gpu_rendered_shards_gather_gloo(mcpt, tmp_path, world, pipeline):
    out = str(tmp_path / "img.npy")
    mp.start_processes(_worker, args=(world, _free_port(), pipeline, out), nprocs=world, start_method="spawn")
    got = np.load(out)
    ref, _ = _single_gpu_image(mcpt, pipeline)
    assert np.array_equal(got[..., :3], ref)


def test_bench_single_process_device_list(mcpt, tmp_path):
    out = str(tmp_path / "img.npy")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--single-process", "--devices", "0,0",
           "--width", str(W), "--height", str(H), "--spp", str(SPP), "--steps", "1", "--warmup", "1",
           "--no-cpu-baseline", "--no-pmc", "--dump-image", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=200, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = _bench_line(r.stdout)
    assert line["n_gpus"] == 2 and "peer-copy gather" in line["config"]["parallelism"]
    got = np.load(out)
    ref, st = _single_gpu_image(mcpt)
    assert np.array_equal(got[..., :3], ref)
    assert line["rays_per_step"] == st["rays"]


def test_bench_gpus_n_without_launcher(mcpt, tmp_path):
    """`python bench.py --gpus 2` with no torch.distributed
    launcher.  With the default RCCL backend on a box with fewer than 2 GPUs it
    exits non-zero and prints no line; under the gloo rehearsal it starts the 2
    ranks itself (a torch.distributed.run child) and prints n_gpus == 2 with
    rank 0's gathered image equal to the one-GPU render."""
    import torch
    base = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--width", str(W), "--height", str(H),
            "--spp", str(SPP), "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-pmc"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MCPT_DIST_BACKEND")}
    if torch.cuda.device_count() < 2:
        r = subprocess.run(base, capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
        assert r.returncode != 0 and "GPU(s) visible" in r.stderr, r.stdout[-2000:] + r.stderr[-2000:]
        assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    out = str(tmp_path / "img.npy")
    r = subprocess.run(base + ["--dump-image", out], capture_output=True, text=True, timeout=280,
                       env=dict(env, MCPT_DIST_BACKEND="gloo"), cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = _bench_line(r.stdout)
    assert line["n_gpus"] == 2 and "x2" in line["config"]["parallelism"]
    ref, st = _single_gpu_image(mcpt)
    assert np.array_equal(np.load(out)[..., :3], ref)
    assert line["rays_per_step"] == st["rays"]
