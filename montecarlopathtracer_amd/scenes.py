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
# QuinEngine's own scene (MCRT/QuinEngine/Res/scene01.{obj,mtl}: the same OBJ,
# its own MTL -- emitter Ka 0.80 without Kd, no Kd/Ka lines on the spheres),
# read by QuinEngine through tinyobjloader (QE/Utils/Structure.hpp:9-12): load
# it with ObjModel(path, flavor="tinyobj").  Unpacked into a subdirectory so
# the files keep their reference names.
BUNDLED_DIRS = {"qe_scene01": ("qe", "scene01")}
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
    sub, base = BUNDLED_DIRS.get(name, ("", name))
    if name not in BUNDLED and name not in BUNDLED_DIRS:
        if os.path.exists(name):
            return name
        raise FileNotFoundError(f"unknown scene {name!r}; bundled: {BUNDLED + tuple(BUNDLED_DIRS)}, "
                                f"generated: {GENERATED}")
    out = os.path.join(_cache_dir(), sub) if sub else _cache_dir()
    os.makedirs(out, exist_ok=True)
    for ext in ("obj", "mtl"):
        dst = os.path.join(out, f"{base}.{ext}")
        src = os.path.join(SCENE_DIR, sub, f"{base}.{ext}.gz")
        if not os.path.exists(dst) or os.path.getmtime(dst) < os.path.getmtime(src):
            with gzip.open(src, "rb") as f:
                data = f.read()
            tmp = dst + f".{os.getpid()}.tmp"
            with open(tmp, "wb") as f:
                f.write(data)
            os.replace(tmp, dst)
    return os.path.join(out, f"{base}.obj")
