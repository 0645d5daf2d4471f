"""C4 workload: the seeded ~70k-triangle mesh in scene01's box.

The generated OBJ is pinned by hash (so every machine renders the same
scene), it goes through the reference-dialect reader, and the KD tree the
product builds on it equals the oracle's restatement of KDTree.hpp node for
node (depth-32 tree, ~1M nodes: the large-scene stress of the build).
"""
import hashlib

import numpy as np

from test_loader_kdtree import _assert_same

MESH_SHA256 = "8e6d62cc9f308fbfd5b59c920fafb8862eeec007844348872b85c452d9754450"


def test_mesh_text_is_pinned(mcpt):
    p = mcpt.scene_path("cornell_bunny70k")
    assert hashlib.sha256(open(p, "rb").read()).hexdigest() == MESH_SHA256


def test_mesh_shape_and_placement():
    from montecarlopathtracer_amd.meshgen import lumpy_sphere, CENTRE, RADIUS
    v, n, t = lumpy_sphere()
    assert t.shape == (70000, 3) and v.shape[0] == 35002
    r = np.linalg.norm(v - np.asarray(CENTRE), axis=1)
    assert r.min() >= 0.8 * RADIUS - 1e-9 and r.max() <= RADIUS + 1e-9
    assert v[:, 1].min() > 0.0                                     # above the floor
    assert np.allclose(np.linalg.norm(n, axis=1), 1.0)
    # outward orientation: face normals point away from the centre
    fn = np.cross(v[t[:, 1]] - v[t[:, 0]], v[t[:, 2]] - v[t[:, 0]])
    fc = v[t].mean(1) - np.asarray(CENTRE)
    assert (np.sum(fn * fc, 1) > 0).mean() > 0.999


def test_mesh_scene_model_and_kd_match_oracle(mcpt, oracle_mod):
    path = mcpt.scene_path("cornell_bunny70k")
    m = mcpt.ObjModel(path)
    g = m.groups()
    assert "pMesh" in g and len(g["pMesh"]) == 70000 and len(g.get("pSphere1", [])) == 0
    _assert_same(mcpt, oracle_mod, path)
    info = mcpt.Scene(m, host_only=True).info()
    assert info["n_triangles"] == 70442 and info["kd_depth"] == 32 and info["lds_bytes"] == 0
