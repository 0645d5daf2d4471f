"""GPU parity on synthetic edge-case scenes, which the reference's own scenes
never hold:

* exactly duplicated triangles carrying different materials -- closest-hit
  ties, decided by (t, rank) in the ordered walk and by the first index in the
  brute force (CUTracer.cu:44-96, strict `t < tmin`);
* degenerate triangles (points and segments) and axis-aligned ones;
* more than 64 coplanar triangles (flat KD nodes, the on-plane rule of
  KDTree.hpp:164-285);
* walls in the planes x = 0 and y = 5 through the eye (0, 5, 17): split planes
  that hold the primary rays' common origin -- the rare branch of the bounce-0
  packet walk and of every lane's step (below / pp by the direction);
* a scene of one triangle.

Each is rendered by both pipelines in both layouts (8-B node image in LDS;
child-box pair records in global memory) against the oracle's ordered walk
(image bit for bit, equal counters) and against its brute force (image bit for
bit: the hits do not depend on the tree)."""
import os

import numpy as np
import pytest

MTL = """newmtl light
Kd 0.8 0.8 0.8
Ka 0.78 0.78 0.78
newmtl diffuse
Kd 0.7 0.5 0.3
newmtl red
Kd 0.9 0.1 0.1
newmtl gloss
Ks 1 1 1
Ns 50
newmtl mirror
Ks 1 1 1
Ns 1000
newmtl glass
Kd 0.5 0.5 0.5
Tr 0.9
Ni 1.5
"""
MATS = ["diffuse", "red", "gloss", "mirror", "glass"]


def _obj(tris, mats):
    lines = ["mtllib t.mtl"]
    for t in tris:
        for p in t:
            lines.append("v %.9g %.9g %.9g" % tuple(p))
    lines.append("vn 0 1 0")
    lines.append("vn 0.6 0.8 0")
    # one group per run of a material, named so that the groups' name order
    # (ObjReader's std::map) is their file order: contiguous geometries
    cur, run = None, 0
    for k, m in enumerate(mats):
        if m != cur:
            lines.append("g g%04d_%s" % (run, m))
            lines.append("usemtl " + m)
            cur, run = m, run + 1
        n = 1 + (k & 1)
        lines.append("f %d//%d %d//%d %d//%d" % (3 * k + 1, n, 3 * k + 2, n, 3 * k + 3, n))
    return "\n".join(lines) + "\n"


def _quad(a, b, c, d):
    return [[a, b, c], [a, c, d]]


def _scene(kind):
    r = np.random.default_rng({"mixed": 11, "flat": 12, "planes": 13, "tiny": 14}[kind])
    tris, mats = [], []

    def add(ts, m):
        for t in ts:
            tris.append(np.asarray(t, np.float64))
            mats.append(m if isinstance(m, str) else m[len(mats) % len(m)])

    if kind == "tiny":
        add([[(-3, 2, 0), (3, 2, 0), (0, 8, 0)]], "light")
    else:
        add(_quad((-6, 10, -6), (6, 10, -6), (6, 10, 6), (-6, 10, 6)), "light")
        add(_quad((-6, 0, -6), (-6, 0, 6), (6, 0, 6), (6, 0, -6)), "diffuse")
        add(_quad((-6, 0, -6), (6, 0, -6), (6, 10, -6), (-6, 10, -6)), "red")
    if kind == "mixed":
        c = r.uniform(-4, 4, (90, 1, 3)) + np.array([0, 5, 0])
        t = c + r.normal(0, 0.7, (90, 3, 3))
        t[:8] = t[:8, :1]                       # points
        t[8:16, 2] = t[8:16, 1]                 # segments
        t[40:60, :, 0] = np.round(t[40:60, :, 0])   # axis-aligned coordinates
        add(t, MATS)
        add(t[20:40], MATS[::-1])               # exact duplicates, other materials (ties)
    elif kind == "flat":
        c = r.uniform(-4, 4, (150, 1, 3))
        t = c + r.normal(0, 0.5, (150, 3, 3))
        t[..., 1] = 3.0                         # >64 coplanar triangles
        add(t, MATS)
        add(t[:10] + np.array([0, 2, 0]), "mirror")
    elif kind == "planes":
        add(_quad((0, 1, -4), (0, 9, -4), (0, 9, 4), (0, 1, 4)), "mirror")       # x = 0 (the eye's x)
        add(_quad((-5, 5, -5), (5, 5, -5), (5, 5, 3), (-5, 5, 3)), "glass")      # y = 5 (the eye's y)
        add(_quad((-3, 2, 0), (3, 2, 0), (3, 8, 0), (-3, 8, 0)), "diffuse")      # z = 0
        c = r.uniform(-4, 4, (40, 1, 3)) + np.array([0, 5, 0])
        add(c + r.normal(0, 0.6, (40, 3, 3)), MATS)
    return np.asarray(tris, np.float32), mats


@pytest.fixture(params=["mixed", "flat", "planes", "tiny"])
def edge_scene(request, tmp_path):
    tris, mats = _scene(request.param)
    (tmp_path / "t.mtl").write_text(MTL)
    p = tmp_path / "t.obj"
    p.write_text(_obj(tris, mats))
    return request.param, str(p)


W, H, SPP, CHUNK = 40, 30, 4, 2
COUNTS = ("rays", "paths", "inner_visits", "leaf_visits", "leaf_refs", "tri_tests", "shades")


def test_edge_scene_oracle_walks_agree(mcpt, oracle_mod, edge_scene):
    """CPU: on these scenes the oracle's ordered walk, its child-box walk and its
    brute force give one image, and the host build lays them out both ways."""
    kind, path = edge_scene
    for layout, boxes in (("auto", 0), ("global", 1)):
        assert mcpt.Scene(mcpt.ObjModel(path), layout=layout, host_only=True).info()["node_boxes"] == boxes
    o = oracle_mod.Scene(path)
    imgs = [o.render(oracle_mod.RenderParams(width=20, height=15, spp=2, threads=4, traversal=t, node_boxes=b))[0]
            for t, b in ((oracle_mod.KD_ORDERED, 0), (oracle_mod.KD_ORDERED, 1), (oracle_mod.BRUTE, 0))]
    assert float(imgs[0].max()) > 0.0, kind
    assert all(np.array_equal(imgs[0].view(np.uint32), x.view(np.uint32)) for x in imgs[1:]), kind


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["auto", "global"])
def test_edge_scene_matches_oracle(mcpt, oracle_mod, edge_scene, layout):
    kind, path = edge_scene
    scene = mcpt.Scene(mcpt.ObjModel(path), layout=layout)
    boxes = scene.info()["node_boxes"]
    assert boxes == (1 if layout == "global" else 0)
    o = oracle_mod.Scene(path)
    threads = min(os.cpu_count() or 8, 16)
    ref, rc = o.render(oracle_mod.RenderParams(width=W, height=H, spp=SPP, spp_chunk=CHUNK, threads=threads,
                                               node_boxes=boxes))
    brute, bc = o.render(oracle_mod.RenderParams(width=W, height=H, spp=SPP, spp_chunk=CHUNK, threads=threads,
                                                 traversal=oracle_mod.BRUTE))
    assert np.array_equal(ref.view(np.uint32), brute.view(np.uint32)), kind   # the oracle's own walks agree
    assert float(ref.max()) > 0.0, kind                                      # the light is seen
    for pipe in ("megakernel", "wavefront"):
        img, st = scene.render(mcpt.RenderParams(width=W, height=H, spp=SPP, spp_chunk=CHUNK, pipeline=pipe))
        assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), (kind, layout, pipe)
        for k in COUNTS:
            assert st[k] == rc[k], (kind, layout, pipe, k, st[k], rc[k])
        for k in ("rays", "paths", "shades"):
            assert st[k] == bc[k], (kind, layout, pipe, k)


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline", ["megakernel", "wavefront", "wavefront-sorted"])
def test_edge_scene_quinengine_mode_matches_oracle(mcpt, oracle_mod, edge_scene, pipeline):
    """The same scenes under rtx.hlsl semantics (roulette, 3x depth cap, QE
    camera and accumulation), LDS layout."""
    kind, path = edge_scene
    depth, seed = 5, 0x5EED
    ref, rc = oracle_mod.Scene(path).render(oracle_mod.RenderParams(
        width=W, height=H, spp=SPP, spp_chunk=CHUNK, max_depth=depth, seed=seed, illum=1.0, fov=45.0,
        fresnel_kd=0, threads=min(os.cpu_count() or 8, 16), mode=oracle_mod.MODE_QE))
    scene = mcpt.Scene(mcpt.ObjModel(path))
    img, st = scene.render(mcpt.RenderParams.for_quinengine(
        width=W, height=H, spp=SPP, spp_chunk=CHUNK, max_depth=depth, seed=seed,
        pipeline="wavefront" if pipeline.startswith("wavefront") else pipeline, wf_sort=pipeline == "wavefront-sorted"))
    assert float(ref.max()) > 0.0, kind
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), (kind, pipeline)
    for k in COUNTS:
        assert st[k] == rc[k], (kind, pipeline, k, st[k], rc[k])


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["auto", "global"])
def test_edge_scene_device_hits(mcpt, oracle_mod, edge_scene, layout):
    """mcpt_intersect on tests/_raysets.py's adversarial families over these
    scenes: the oracle walk's hits and counters bit for bit, and the brute
    force's off the triangle-edge origins (family 5)."""
    import warnings
    from _raysets import ray_sets
    kind, path = edge_scene
    if kind == "tiny":
        pytest.skip("one leaf, no split planes for family 4")
    scene = mcpt.Scene(mcpt.ObjModel(path), layout=layout)
    boxes = int(scene.info()["node_boxes"])
    o_s = oracle_mod.Scene(path)
    n = 40_000
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)     # point triangles: zero directions, dropped
        o, d = ray_sets(o_s, n, seed=29)
    tri, hit, st = scene.intersect(o, d)
    tk, _, hk, ck = o_s.intersect(o, d, oracle_mod.KD_ORDERED, node_boxes=boxes, threads=8)
    assert np.array_equal(tri, tk)
    hit_k = np.where(tk[:, None] >= 0, hk[:, :3], 0.0).astype(np.float32)
    hit_g = np.where(tri[:, None] >= 0, hit, 0.0).astype(np.float32)
    assert np.array_equal(hit_g.view(np.uint32), hit_k.view(np.uint32))
    for k in ("inner_visits", "leaf_visits", "leaf_refs", "tri_tests"):
        assert st[k] == ck[k], (k, st[k], ck[k])
    tb, _, hb, _ = o_s.intersect(o, d, oracle_mod.BRUTE, threads=8)
    k5 = n // 8
    fam5 = np.zeros(o.shape[0], bool)
    fam5[6 * k5:7 * k5] = True
    bad = np.nonzero((tb != tri) | (np.where(tb[:, None] >= 0, hb[:, :3], 0.0).astype(np.float32).view(np.uint32)
                                    != hit_g.view(np.uint32)).any(axis=1))[0]
    assert not (~fam5[bad]).any(), bad[~fam5[bad]][:10]
    assert (tri >= 0).mean() > 0.3
