"""Bundled scene assets.

The reference ships its Cornell-box scenes as OBJ/MTL text
(CVMCTracer/CVMCTracer/Resources/scene0{1,2,3}.{obj,mtl}); they are bundled
here gzip-compressed and unpacked on demand into a cache directory, because
the loaders (like the reference's ``ObjModel::readObj(path)``,
ObjReader.cpp:8) take a file path.
"""
from __future__ import annotations

import gzip
import os
import tempfile

_HERE = os.path.dirname(os.path.abspath(__file__))
SCENE_DIR = os.path.join(_HERE, "scenes")
BUNDLED = ("scene01", "scene02", "scene03")
GENERATED = ("cornell_bunny70k",)   # meshgen.cornell_mesh_scene (C4 workload)


def _cache_dir() -> str:
    d = os.environ.get("MCPT_SCENE_CACHE") or os.path.join(tempfile.gettempdir(), f"mcpt_scenes_{os.getuid()}")
    os.makedirs(d, exist_ok=True)
    return d


def scene_path(name: str) -> str:
    """Return a filesystem path to ``<name>.obj`` (with its .mtl beside it)."""
    if name in GENERATED:
        from .meshgen import cornell_mesh_scene
        return cornell_mesh_scene(name)
    if name not in BUNDLED:
        if os.path.exists(name):
            return name
        raise FileNotFoundError(f"unknown scene {name!r}; bundled: {BUNDLED}, generated: {GENERATED}")
    out = _cache_dir()
    for ext in ("obj", "mtl"):
        dst = os.path.join(out, f"{name}.{ext}")
        src = os.path.join(SCENE_DIR, f"{name}.{ext}.gz")
        if not os.path.exists(dst) or os.path.getmtime(dst) < os.path.getmtime(src):
            with gzip.open(src, "rb") as f:
                data = f.read()
            tmp = dst + f".{os.getpid()}.tmp"
            with open(tmp, "wb") as f:
                f.write(data)
            os.replace(tmp, dst)
    return os.path.join(out, f"{name}.obj")
