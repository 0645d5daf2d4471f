"""Device closest-hit queries (mcpt_intersect: the render traversal run on
caller-given rays) against the CPU oracle on the adversarial ray families of
tests/_raysets.py -- origins exactly on KD split planes, axis-parallel and
grazing rays, origins on triangle edges, rays through vertices.

Held bit for bit (triangle id, beta, gamma, t) and counter for counter to the
oracle's ordered walk with the same child-box cull the scene's layout uses
(scene01 in LDS: no boxes; scenes 02/03 and the C4 mesh from global memory:
fp16 child boxes), and -- except where an origin sits on a triangle edge, which
tests/test_brute_pins.py shows to be float artifacts of the reference's own
arithmetic -- to the brute force of CUTracer.cu:44-96.
"""
import numpy as np
import pytest

from _raysets import ray_sets

pytestmark = pytest.mark.gpu

N = 100_000


@pytest.mark.parametrize("name", ["scene01", "scene02", "scene03", "cornell_bunny70k"])
def test_device_hits_equal_oracle_walk_and_brute_force(mcpt, oracle_mod, name):
    path = mcpt.scene_path(name)
    scene = mcpt.Scene(mcpt.ObjModel(path))
    boxes = int(scene.info()["node_boxes"])
    o_s = oracle_mod.Scene(path)
    o, d = ray_sets(o_s, N, seed=23)
    tri, hit, st = scene.intersect(o, d)
    tk, gk, hk, ck = o_s.intersect(o, d, oracle_mod.KD_ORDERED, node_boxes=boxes, threads=8)
    assert np.array_equal(tri, tk)
    hit_k = np.where(tk[:, None] >= 0, hk[:, :3], 0.0).astype(np.float32)
    hit_g = np.where(tri[:, None] >= 0, hit, 0.0).astype(np.float32)
    assert np.array_equal(hit_g.view(np.uint32), hit_k.view(np.uint32))
    assert st["rays"] == o.shape[0]
    for k in ("inner_visits", "leaf_visits", "leaf_refs", "tri_tests"):
        assert st[k] == ck[k], (k, st[k], ck[k])
    # brute force: equal off the triangle-edge origins (family 5)
    tb, gb, hb, _ = o_s.intersect(o, d, oracle_mod.BRUTE, threads=8)
    k5 = N // 8
    fam5 = np.zeros(o.shape[0], bool)
    fam5[6 * k5:7 * k5] = True
    bad = np.nonzero((tb != tri) | (np.where(tb[:, None] >= 0, hb[:, :3], 0.0).astype(np.float32).view(np.uint32)
                                    != hit_g.view(np.uint32)).any(axis=1))[0]
    assert not (~fam5[bad]).any(), bad[~fam5[bad]][:10]
    assert 0.3 < (tri >= 0).mean() < 1.0


def test_intersect_t_max_and_empty(mcpt, oracle_mod):
    """t_max bounds the closest hit (QuinEngine's t_best = 10000, rtx.hlsl:88); n = 0 is a no-op."""
    path = mcpt.scene_path("scene01")
    scene = mcpt.Scene(mcpt.ObjModel(path))
    # (the eye's axis ray through (0, 5) would run along the back wall quad's
    # diagonal, which the strict Cramer test of CUTracer.cu:86 rejects on both sides)
    o = np.tile(np.array([[0.1, 5.1, 17.0]], np.float32), (64, 1))
    d = np.tile(np.array([[0.01, 0.02, -1.0]], np.float32), (64, 1))
    tri, hit, _ = scene.intersect(o, d)
    assert (tri >= 0).all() and (hit[:, 2] > 1.0).all()
    t0 = float(hit[0, 2])
    tri2, _, _ = scene.intersect(o, d, t_max=t0 * 0.5)
    assert (tri2 == -1).all()
    tri3, hit3, st = scene.intersect(np.zeros((0, 3), np.float32), np.zeros((0, 3), np.float32))
    assert tri3.size == 0 and st["rays"] == 0
