"""The opt-in SAH KD tree (mcpt_scene_options::kd_build = MCPT_KD_BUILD_SAH) on
the GPU: both pipelines render the oracle's image bit for bit with equal
counters when the oracle walks the same tree (oracle/kdtree_ref.c sah_split),
and -- the closest hit being the brute-force (t, rank) minimum for any tree --
the reference tree's image too, with fewer node visits.  Scenes in LDS
(scene01, scene02), the global layout with the child-box cull (scene01 forced
global, the C4 mesh), and a C2 crop at its own 1024 spp.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = [
    # scene, W, H, spp, chunk, layout
    ("scene01", 64, 48, 8, 4, "auto"),
    ("scene02", 48, 36, 4, 2, "auto"),
    ("scene03", 40, 30, 4, 4, "auto"),
    ("scene01", 48, 40, 6, 3, "global"),
    ("cornell_bunny70k", 40, 32, 4, 2, "auto"),
]
KEYS = ("rays", "paths", "inner_visits", "leaf_visits", "leaf_refs", "tri_tests", "shades")


@pytest.mark.parametrize("pipeline", ["megakernel", "wavefront"])
@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-{c[5]}-{c[1]}x{c[2]}" for c in CASES])
def test_sah_tree_matches_oracle_and_reference_tree_image(mcpt, oracle_mod, case, pipeline):
    sc, W, H, spp, chunk, layout = case
    path = mcpt.scene_path(sc)
    scene_id = 2 if sc in ("scene02", "scene03") else 1
    scene = mcpt.Scene(mcpt.ObjModel(path), layout=layout, kd_build="sah")
    info = scene.info()
    assert info["kd_build"] == 1
    p = mcpt.RenderParams.for_scene(scene_id, width=W, height=H, spp=spp, spp_chunk=chunk, pipeline=pipeline)
    img, st = scene.render(p)
    o = oracle_mod.Scene(path, kd_build="sah")
    ref, rc = o.render(oracle_mod.RenderParams(width=W, height=H, spp=spp, spp_chunk=chunk, scene_id=scene_id,
                                               traversal=oracle_mod.KD_ORDERED, threads=8,
                                               node_boxes=info["node_boxes"]))
    assert np.array_equal(img, ref), f"max abs diff {np.abs(img - ref).max()}"
    for k in KEYS:
        assert st[k] == rc[k], (k, st[k], rc[k])
    # the reference tree's render: the same image, more node visits on the LDS scenes
    base, sb = mcpt.Scene(mcpt.ObjModel(path), layout=layout).render(p)
    assert np.array_equal(img.view(np.uint32), base.view(np.uint32))
    assert st["rays"] == sb["rays"]
    if layout == "auto" and sc in ("scene01", "scene02"):
        assert st["inner_visits"] < (0.75 if sc == "scene01" else 1.0) * sb["inner_visits"]


def test_sah_tree_c2_crop_full_spp(mcpt, oracle_mod):
    """A 32x32 crop of the C2 frame (1024^2, 1024 spp) on the wavefront
    pipeline, lean, with the SAH tree: the oracle's crop bit for bit."""
    path = mcpt.scene_path("scene01")
    scene = mcpt.Scene(mcpt.ObjModel(path), kd_build="sah")
    x0, y0, n = 496, 560, 32
    p = mcpt.RenderParams(width=1024, height=1024, spp=1024, spp_chunk=32, pipeline="wavefront")
    img, st = scene.render(p)
    o = oracle_mod.Scene(path, kd_build="sah")
    ref, _ = o.render(oracle_mod.RenderParams(width=1024, height=1024, spp=1024, spp_chunk=32,
                                              traversal=oracle_mod.KD_ORDERED, threads=8,
                                              region=(x0, y0, x0 + n, y0 + n)))
    assert np.array_equal(img[y0:y0 + n, x0:x0 + n], ref[y0:y0 + n, x0:x0 + n])
