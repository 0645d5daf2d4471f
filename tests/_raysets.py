"""Adversarial ray families for closest-hit pins (tests/test_brute_pins.py on
the CPU oracle, tests/test_gpu_intersect.py on the device): random rays, rays
aimed at triangle interiors, axis-parallel rays, origins exactly on KD split
planes, origins on triangle edges (family 5: indices [6k, 7k), k = n // 8),
rays grazing a triangle's plane and rays through vertices."""
import numpy as np


def ray_sets(s, n, seed):
    """n rays (origins, directions float32) over the scene's root box in seven families."""
    r = np.random.default_rng(seed)
    nodes = s.kd_nodes()
    bmin, bmax = nodes[0, 4:7].view(np.float32), nodes[0, 7:10].view(np.float32)
    ext = bmax - bmin
    kv = s.kd_verts()                                     # (nkd, 3, 3) float32
    k = n // 8

    def unit(v):
        v = v.astype(np.float64)
        return (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)

    def in_box(m):
        return (bmin + ext * r.random((m, 3))).astype(np.float32)

    def tri_points(m, tris=None):
        t = r.integers(0, kv.shape[0], m) if tris is None else tris
        a, b = r.random(m), r.random(m)
        sw = a + b > 1
        a[sw], b[sw] = 1 - a[sw], 1 - b[sw]
        v = kv[t].astype(np.float64)
        return (v[:, 0] + a[:, None] * (v[:, 1] - v[:, 0]) + b[:, None] * (v[:, 2] - v[:, 0])).astype(np.float32), t

    O, D = [], []
    # 1 random rays
    O.append(in_box(2 * k)); D.append(unit(r.standard_normal((2 * k, 3))))
    # 2 aimed at triangle interiors
    o = in_box(2 * k); p, _ = tri_points(2 * k)
    O.append(o); D.append(unit(p - o))
    # 3 axis-parallel: one or two zero components (the dir == 0 slab paths)
    d = r.standard_normal((k, 3))
    z = r.integers(0, 3, k)
    d[np.arange(k), z] = 0.0
    two = r.random(k) < 0.5
    d[np.arange(k)[two], (z[two] + 1) % 3] = 0.0
    O.append(in_box(k)); D.append(unit(d))
    # 4 origins exactly on KD split planes, inside the node's box
    inner = np.nonzero(nodes[:, 2])[0]
    pick = inner[r.integers(0, inner.size, k)]
    nb0, nb1 = nodes[pick, 4:7].view(np.float32), nodes[pick, 7:10].view(np.float32)
    o = (nb0 + (nb1 - nb0) * r.random((k, 3))).astype(np.float32)
    ax = nodes[pick, 2].astype(np.int64) - 1
    o[np.arange(k), ax] = nodes[pick, 3].view(np.float32)
    half = k // 2
    p, _ = tri_points(k)
    d = unit(r.standard_normal((k, 3)))
    d[:half] = unit(p[:half] - o[:half])
    O.append(o); D.append(d)
    # 5 origins on triangle edges; half toward the opposite vertex (in the triangle's plane)
    t = r.integers(0, kv.shape[0], k)
    e = r.integers(0, 3, k)
    a = kv[t, e].astype(np.float64); b = kv[t, (e + 1) % 3].astype(np.float64); c = kv[t, (e + 2) % 3]
    o = (a + r.random((k, 1)) * (b - a)).astype(np.float32)
    d = unit(r.standard_normal((k, 3)))
    d[:half] = unit(c[:half].astype(np.float64) - o[:half])
    O.append(o); D.append(d)
    # 6 grazing: in the plane of a triangle (direction along one of its edges), origin
    #   a tiny distance off the plane or on it, aimed across the triangle
    t = r.integers(0, kv.shape[0], k)
    v = kv[t].astype(np.float64)
    nrm = np.cross(v[:, 1] - v[:, 0], v[:, 2] - v[:, 0])
    nrm /= np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-30)
    cen = v.mean(axis=1)
    edge = v[:, 1] - v[:, 0]
    off = r.choice([0.0, 1e-6, -1e-6, 1e-4], size=(k, 1))
    o = (cen - 2.0 * edge + off * nrm).astype(np.float32)
    O.append(o); D.append(unit(edge))
    # 7 through vertices
    rest = n - sum(x.shape[0] for x in O)
    o = in_box(rest)
    vv = kv[r.integers(0, kv.shape[0], rest), r.integers(0, 3, rest)]
    O.append(o); D.append(unit(vv.astype(np.float64) - o))
    O, D = np.concatenate(O), np.concatenate(D)
    ok = np.isfinite(D).all(axis=1) & (np.abs(D).sum(axis=1) > 0)
    return O[ok], D[ok]
