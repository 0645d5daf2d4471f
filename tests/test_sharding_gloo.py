"""Multi-rank path (N > 1) on CPU: two gloo ranks shard an image into
interleaved tiles, 'render' their tiles (slices of an oracle image, standing in
for the GPU path) and TileGather reassembles the full image on rank 0 -- the
same code bench.py runs over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, W, H, image, out_path):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import montecarlopathtracer_amd as M
    from montecarlopathtracer_amd.sharding import TileGather, shard_params
    base = M.RenderParams(width=W, height=H, spp=1)
    p = shard_params(base, world, rank)
    xy = p.shard_pixels()
    local = np.zeros((xy.shape[0], 4), np.float32)
    ok = xy[:, 0] >= 0
    local[ok, :3] = image[xy[ok, 1], xy[ok, 0]]
    g = TileGather(W, H, world, rank, torch.device("cpu"))
    out = g.gather(torch.from_numpy(local))
    if rank == 0:
        np.save(out_path, out.numpy())
    dist.destroy_process_group()


def _finish_worker(rank, world, port, out_dir):
    import datetime
    import importlib.util
    import time
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=2))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("_bench", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    if rank == 0:
        time.sleep(5)          # rank 0's untimed post-processing, longer than the group's timeout
    bench.finish_ranks(dist, rank, datetime)
    with open(os.path.join(out_dir, f"r{rank}"), "w") as f:
        f.write(str(time.time()))
    dist.destroy_process_group()


def test_bench_ranks_wait_for_rank0_line():
    """bench.finish_ranks: ranks 1..N-1 outwait rank 0's post-timing work (a
    collective would time out after the group's 2 s here) and tear down with it."""
    import tempfile
    import time
    with tempfile.TemporaryDirectory() as d:
        t0 = time.time()
        mp.start_processes(_finish_worker, args=(3, _free_port(), d), nprocs=3, start_method="spawn")
        ends = [float(open(os.path.join(d, f"r{r}")).read()) for r in range(3)]
    assert min(ends) - t0 >= 5.0 and max(ends) - min(ends) < 2.0


@pytest.mark.parametrize("W,H", [(64, 40), (37, 29)])
def test_tile_gather_reassembles_image_gloo(oracle_mod, tmp_path, W, H):
    from montecarlopathtracer_amd.scenes import scene_path
    s = oracle_mod.Scene(scene_path("scene01"))
    image, _ = s.render(oracle_mod.RenderParams(width=W, height=H, spp=2, threads=4))
    out_path = str(tmp_path / "img.npy")
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), W, H, image, out_path), nprocs=world,
                       start_method="spawn")
    got = np.load(out_path).reshape(H, W, 4)
    assert np.array_equal(got[..., :3], image)
