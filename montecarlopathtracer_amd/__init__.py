"""montecarlopathtracer_amd -- MI355X-native Monte Carlo path-tracing core.

A drop-in for the hot path of pw1316/MonteCarloPathTracer (the CVMCTracer
per-pixel megakernel with the QuinEngine KD tree): OBJ/MTL scene load, KD
build, and a hand-written HIP/gfx950 path kernel behind the C ABI in
include/mcpt.h.  See DESIGN.md and INTEGRATION.md.

Importing this package loads lib/libmcpt.so; there is no CPU fallback.
"""
from ._capi import McptError, lib  # noqa: F401  (loads libmcpt.so, raises if missing)
from .imageio import read_pfm, read_png, write_pfm, write_png
from .scenes import scene_path
from .tracer import (ILLUM, IMG_HEIGHT, IMG_WIDTH, NUM_KERNELS, NUM_SAMPLES_PER_KERNEL, CreateGeometry,
                     DestroyGeometry, Initialize, ObjModel, RenderParams, RenderScene, Scene, Tracer, encode_8bit)

lib()

__all__ = ["McptError", "ObjModel", "RenderParams", "Scene", "Tracer", "Initialize", "CreateGeometry",
           "DestroyGeometry", "RenderScene", "encode_8bit", "scene_path", "IMG_WIDTH", "IMG_HEIGHT",
           "NUM_KERNELS", "NUM_SAMPLES_PER_KERNEL", "ILLUM", "write_png", "read_png", "write_pfm", "read_pfm"]
