"""Deterministic large-mesh scenes for the C4 configuration.

There is no Stanford bunny in the reference (nor network access to fetch
one), so C4 uses a seeded ~70k-triangle "lumpy sphere" placed where pSphere1
sits in scene01 (radius 1.6, centre (-2.37, 1.6, -1.56)): the Cornell box of
scene01 with pSphere1's faces replaced by the mesh.  The output is plain OBJ
+ MTL text in the reference's dialect (groups, usemtl, ``f v/vt/vn``), so the
whole path -- ObjModel::readObj (ObjReader.cpp:8-161), CreateGeometry
(CUTracer.cu:225-314), the KD build (KDTree.hpp:58-287) and the kernel --
runs on it unchanged.

The mesh is a UV sphere with ``slices`` x ``stacks`` cells (2*slices*(stacks-1)
triangles) whose radius is modulated by seeded Gaussian bumps and low-order
spherical waves; vertex normals are area-weighted face-normal averages.
Everything is numpy float64 arithmetic formatted with '%.6f', so the text
(and its hash) is identical on every machine.
"""
from __future__ import annotations

import hashlib
import os

import numpy as np

from .scenes import _cache_dir, scene_path

CENTRE = (-2.37, 1.6, -1.56)   # pSphere1 in scene01.obj
RADIUS = 1.6


def lumpy_sphere(slices: int = 200, stacks: int = 176, seed: int = 0x4D435054, radius: float = RADIUS,
                 centre=CENTRE):
    """Returns (verts (V,3), normals (V,3), tris (F,3) 0-based) of the seeded mesh."""
    rng = np.random.default_rng(seed)
    theta = np.pi * np.arange(1, stacks) / stacks                 # ring polar angles
    phi = 2.0 * np.pi * np.arange(slices) / slices
    th, ph = np.meshgrid(theta, phi, indexing="ij")
    dirs = np.stack([np.sin(th) * np.cos(ph), np.cos(th), np.sin(th) * np.sin(ph)], -1).reshape(-1, 3)
    dirs = np.concatenate([[[0.0, 1.0, 0.0]], dirs, [[0.0, -1.0, 0.0]]], 0)
    # radius modulation in [0.80, 1.0] * radius: bumps + waves, never below the floor
    nb = 24
    c = rng.normal(size=(nb, 3))
    c /= np.linalg.norm(c, axis=1, keepdims=True)
    amp = rng.uniform(-0.5, 1.0, nb)
    width = rng.uniform(0.25, 0.7, nb)
    g = np.exp(-np.sum((dirs[:, None, :] - c[None]) ** 2, -1) / (width[None] ** 2)) @ amp
    f = rng.uniform(2.0, 7.0, (6, 3))
    ph0 = rng.uniform(0, 2 * np.pi, (6, 3))
    w = sum(np.prod(np.sin(f[k][None] * dirs * np.pi + ph0[k][None]), -1) for k in range(6))
    m = g + 0.35 * w
    m = (m - m.min()) / (m.max() - m.min())
    r = radius * (0.80 + 0.20 * m)
    verts = dirs * r[:, None] + np.asarray(centre)[None]

    S, T = slices, stacks
    ring = lambda i: 1 + i * S                                      # first vertex of ring i (0..T-2)
    tris = []
    j = np.arange(S)
    jn = (j + 1) % S
    tris.append(np.stack([np.zeros(S, int), ring(0) + jn, ring(0) + j], -1))            # top cap
    for i in range(T - 2):
        a, b = ring(i) + j, ring(i) + jn
        cc, d = ring(i + 1) + j, ring(i + 1) + jn
        tris.append(np.stack([a, b, d], -1))
        tris.append(np.stack([a, d, cc], -1))
    last = 1 + (T - 1) * S
    tris.append(np.stack([np.full(S, last), ring(T - 2) + j, ring(T - 2) + jn], -1))    # bottom cap
    tris = np.concatenate(tris, 0)

    fn = np.cross(verts[tris[:, 1]] - verts[tris[:, 0]], verts[tris[:, 2]] - verts[tris[:, 0]])
    nrm = np.zeros_like(verts)
    for k in range(3):
        np.add.at(nrm, tris[:, k], fn)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    return verts, nrm, tris


def cornell_mesh_scene(name: str = "cornell_bunny70k", slices: int = 200, stacks: int = 176,
                       seed: int = 0x4D435054) -> str:
    """Write (once) and return the path of scene01 with pSphere1 replaced by the mesh."""
    base = scene_path("scene01")
    key = hashlib.sha1(f"{slices}:{stacks}:{seed}:v1".encode()).hexdigest()[:10]
    out = os.path.join(_cache_dir(), f"{name}_{key}.obj")
    if os.path.exists(out):
        return out
    src = open(base).read().splitlines()
    mtl = open(os.path.splitext(base)[0] + ".mtl").read()
    nv = sum(1 for l in src if l.startswith("v "))
    nvt = sum(1 for l in src if l.startswith("vt "))
    nvn = sum(1 for l in src if l.startswith("vn "))
    lines, group = [], None
    for l in src:
        if l.startswith("g "):
            group = l[2:].strip()
        if l.startswith("mtllib"):
            l = f"mtllib {os.path.basename(out)[:-4]}.mtl"
        if group == "pSphere1" and l.startswith("f "):
            continue                                              # drop the sphere's faces
        lines.append(l)
    v, n, t = lumpy_sphere(slices, stacks, seed)
    lines.append("g default")
    lines += ["v %.6f %.6f %.6f" % tuple(p) for p in v]
    lines.append("vt 0.500000 0.500000")
    lines += ["vn %.6f %.6f %.6f" % tuple(p) for p in n]
    lines.append("s 1")
    lines.append("g pMesh")
    lines.append("usemtl mesh_diffuse")
    vt = nvt + 1
    lines += ["f %d/%d/%d %d/%d/%d %d/%d/%d" % (nv + a + 1, vt, nvn + a + 1, nv + b + 1, vt, nvn + b + 1,
                                                  nv + c + 1, vt, nvn + c + 1) for a, b, c in t]
    mtl += "newmtl mesh_diffuse\nillum 4\nKd 0.75 0.72 0.65\nKa 0.00 0.00 0.00\n"
    tmp = out + f".{os.getpid()}.tmp"
    with open(os.path.splitext(out)[0] + ".mtl", "w") as f:
        f.write(mtl)
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, out)
    return out
