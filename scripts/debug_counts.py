"""Diagnostics: locate pixels whose GPU traversal counters differ from the oracle."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle
import montecarlopathtracer_amd as M

W, H, spp, chunk = 64, 48, 8, 4
path = M.scene_path("scene01")
scene = M.Scene(M.ObjModel(path))
p = M.RenderParams(width=W, height=H, spp=spp, spp_chunk=chunk, tile=8)
fb, uc = scene.render_unit_counters(p)
xy = p.shard_pixels() if p.packed else None
npix = W * H
# unit u = chunk*npix_local + v ; v in tile order (tile=8)
pk = M.RenderParams(width=W, height=H, spp=spp, spp_chunk=chunk, tile=8, packed=True).shard_pixels()
per_v = uc.reshape(-1, len(pk), 4).sum(axis=0)
o = oracle.Scene(path)
bad = 0
for v in range(len(pk)):
    x, y = pk[v]
    if x < 0:
        continue
    op = oracle.RenderParams(width=W, height=H, spp=spp, spp_chunk=chunk, region=(x, y, x + 1, y + 1))
    _, c = o.render(op)
    oc = [c["rays"], c["inner_visits"], c["leaf_visits"], c["tri_tests"]]
    if list(per_v[v]) != oc:
        bad += 1
        print("pixel", x, y, "gpu", list(per_v[v]), "oracle", oc)
print("bad pixels", bad)
