"""Pixel-tile sharding across GPUs and the tile gather to rank 0.

The image is cut into tile x tile pixel tiles; tile t belongs to rank
t % world (interleaved, so every rank gets a similar mix of the bright floor,
the spheres and the ~20% black miss region).  Each rank renders its tiles
packed (mcpt_render_params.packed) into a (n_local, 4) float buffer; rank 0
gathers every rank's buffer with one torch.distributed.gather (RCCL over xGMI
on MI355X, gloo on CPU) and scatters the slots back to image order.

There is no reference counterpart: the reference renders on one device
(CUTracer.cu:220-223 selects device 0).
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np

from .tracer import RenderParams


def shard_params(base: RenderParams, world: int, rank: int, tile: int = 8) -> RenderParams:
    """Copy of base restricted to rank's tiles, written packed."""
    import dataclasses
    return dataclasses.replace(base, tile=tile, shard_count=world, shard_index=rank, packed=world > 1)


class TileGather:
    """Gathers packed per-rank tile buffers into one row-major (H*W, 4) image on rank 0."""

    def __init__(self, width: int, height: int, world: int, rank: int, device, tile: int = 8):
        import torch
        self.width, self.height, self.world, self.rank, self.tile = width, height, world, rank, tile
        probe = [RenderParams(width=width, height=height, tile=tile, shard_count=world, shard_index=r)
                 for r in range(world)]
        self.counts: List[int] = [p.output_pixels() for p in probe]
        self.maxn = max(self.counts)
        self.n_local = self.counts[rank]
        self.send = torch.zeros((self.maxn, 4), dtype=torch.float32, device=device)
        self.recv = None
        self.image = None
        if rank == 0:
            # one contiguous receive buffer (rank r's slots at r * maxn) and one
            # precomputed slot -> pixel map: the unpermute is a single gather
            # kernel with no host synchronisation
            self.recv_all = torch.zeros((world * self.maxn, 4), dtype=torch.float32, device=device)
            self.recv = list(self.recv_all.view(world, self.maxn, 4).unbind(0))
            self.image = torch.zeros((height * width, 4), dtype=torch.float32, device=device)
            src, dst = [], []
            for r in range(world):
                xy = probe[r].shard_pixels().astype(np.int64)
                ok = np.nonzero(xy[:, 0] >= 0)[0]
                src.append(r * self.maxn + ok)
                dst.append(xy[ok, 1] * width + xy[ok, 0])
            self.src = torch.from_numpy(np.concatenate(src)).to(device)
            self.dst = torch.from_numpy(np.concatenate(dst)).to(device)

    def gather(self, fb_local) -> Optional["torch.Tensor"]:
        """fb_local: (n_local, 4) packed tiles of this rank. Returns the image on rank 0, None elsewhere."""
        import torch.distributed as dist
        self.send[: self.n_local].copy_(fb_local[: self.n_local])
        if self.send.is_cuda and dist.get_backend() == "gloo":
            # gloo has no device gather: stage through host memory (single-box rehearsal only)
            recv = [r.cpu() for r in self.recv] if self.rank == 0 else None
            dist.gather(self.send.cpu(), recv, dst=0)
            if self.rank == 0:
                for d, h in zip(self.recv, recv):
                    d.copy_(h)
        else:
            dist.gather(self.send, self.recv if self.rank == 0 else None, dst=0)
        if self.rank != 0:
            return None
        self.image.index_copy_(0, self.dst, self.recv_all.index_select(0, self.src))
        return self.image
