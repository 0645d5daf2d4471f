"""Host-side mirror of the reference tracer interface, over the C ABI.

Reference interface (pw1316/MonteCarloPathTracer, CVMCTracer/CVMCTracer):
  PW::FileReader::ObjModel::readObj(path)        Framework/ObjReader.hpp:55
  PW::Tracer::Initialize()                       CUDA/CUTracer.h:9
  PW::Tracer::CreateGeometry(const ObjModel*)    CUDA/CUTracer.h:10
  PW::Tracer::DestroyGeometry()                  CUDA/CUTracer.h:11
  PW::Tracer::RenderScene(sceneID, hostcolor)    CUDA/CUTracer.h:12
and its only caller, main.cpp:16-18 / 33-35.

Same names, argument meaning and call order.  Differences:
  * errors raise McptError instead of returning a mostly-ignored cudaError_t;
  * the scene is held by a Tracer object (module functions keep one default
    Tracer, like the reference's module globals);
  * RenderScene keeps the reference's progressive loop (NUM_KERNELS launches of
    NUM_SAMPLES_PER_KERNEL samples, running mean with prevCount, CUTracer.cu:
    378-398) but without the OpenCV window/PNG side effects.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

from . import _capi
from ._capi import McptError, RenderParamsC, RenderStats, check, lib

# CV/stdafx.h:41-46
IMG_WIDTH = 800
IMG_HEIGHT = 600
NUM_KERNELS = 100
NUM_SAMPLES_PER_KERNEL = 100
ILLUM = 10.0
DEFAULT_SEED = 0x4D435054


def _fptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class ObjModel:
    """PW::FileReader::ObjModel (ObjReader.hpp:37-63): OBJ/MTL data with dummy index 0."""

    FLAVORS = {"cvmctracer": _capi.OBJ_CVMCTRACER, "tinyobj": _capi.OBJ_TINYOBJ}

    def __init__(self, path: Optional[str] = None, flavor: str = "cvmctracer"):
        """flavor "tinyobj": read as QuinEngine does through tinyobjloader
        (mcpt_model_read_obj_ex, include/mcpt.h) -- use it for qe_scene01."""
        self._h = None
        self.path = None
        if path is not None:
            self.read_obj(path, flavor)

    def read_obj(self, path: str, flavor: str = "cvmctracer") -> bool:   # ObjModel::readObj (ObjReader.cpp:8)
        if flavor not in self.FLAVORS:
            raise ValueError(f"flavor must be one of {sorted(self.FLAVORS)}")
        h = C.c_void_p()
        check(lib().mcpt_model_read_obj_ex(path.encode(), self.FLAVORS[flavor], C.byref(h)))
        self._free()
        self._h = h
        self.path = path
        return True

    readObj = read_obj

    @classmethod
    def from_arrays(cls, vertices, normals, triangles, materials, groups: dict) -> "ObjModel":
        """Build from in-memory arrays laid out like ObjReader.hpp:57-63 (element 0 = dummy):
        vertices (n,3), normals (n,3), triangles (n,10) v/t/n/material, materials (n,12)
        Ka Kd Ks Ns Tr Ni, groups {name: triangle indices}."""
        v = np.ascontiguousarray(vertices, np.float32)
        n = np.ascontiguousarray(normals, np.float32)
        t = np.ascontiguousarray(triangles, np.int32)
        m = np.ascontiguousarray(materials, np.float64)
        names = list(groups)
        offs = np.zeros(len(names) + 1, np.int64)
        for i, k in enumerate(names):
            offs[i + 1] = offs[i] + len(groups[k])
        gt = np.ascontiguousarray(np.concatenate([np.asarray(groups[k], np.int32) for k in names])
                                  if names else np.zeros(0, np.int32), np.int32)
        cnames = (C.c_char_p * max(len(names), 1))(*[k.encode() for k in names])
        d = _capi.ModelDesc()
        d.vertices, d.n_vertices = v.ctypes.data_as(C.POINTER(C.c_float)), v.shape[0]
        d.normals, d.n_normals = n.ctypes.data_as(C.POINTER(C.c_float)), n.shape[0]
        d.triangles, d.n_triangles = t.ctypes.data_as(C.POINTER(C.c_int32)), t.shape[0]
        d.materials, d.n_materials = m.ctypes.data_as(C.POINTER(C.c_double)), m.shape[0]
        d.group_names, d.group_offsets = cnames, offs.ctypes.data_as(C.POINTER(C.c_int64))
        d.group_tris, d.n_groups = gt.ctypes.data_as(C.POINTER(C.c_int32)), len(names)
        h = C.c_void_p()
        check(lib().mcpt_model_create(C.byref(d), C.byref(h)))
        obj = cls()
        obj._h = h
        obj.path = "<memory>"
        return obj

    def _free(self):
        if self._h is not None and _capi._lib is not None:
            _capi._lib.mcpt_model_free(self._h)
        self._h = None

    def __del__(self):
        self._free()

    @property
    def handle(self):
        if self._h is None:
            raise McptError(-1, "model not loaded")
        return self._h

    def info(self) -> dict:
        i = _capi.ModelInfo()
        check(lib().mcpt_model_get_info(self.handle, C.byref(i)))
        return {n: int(getattr(i, n)) for n, _ in i._fields_}

    def vertices(self) -> np.ndarray:
        a = np.zeros((self.info()["n_vertices"], 3), np.float32)
        check(lib().mcpt_model_copy_vertices(self.handle, _fptr(a)))
        return a

    def normals(self) -> np.ndarray:
        a = np.zeros((self.info()["n_normals"], 3), np.float32)
        check(lib().mcpt_model_copy_normals(self.handle, _fptr(a)))
        return a

    def triangles(self) -> np.ndarray:
        """(n, 10) int32: vertex[3], texture[3], normal[3], material index."""
        a = np.zeros((self.info()["n_triangles"], 10), np.int32)
        check(lib().mcpt_model_copy_triangles(self.handle, a.ctypes.data_as(C.POINTER(C.c_int32))))
        return a

    def materials(self) -> np.ndarray:
        """(n, 12) float64: Ka[3] Kd[3] Ks[3] Ns Tr Ni."""
        a = np.zeros((self.info()["n_materials"], 12), np.float64)
        check(lib().mcpt_model_copy_materials(self.handle, a.ctypes.data_as(C.POINTER(C.c_double))))
        return a

    def groups(self) -> dict:
        out = {}
        buf = C.create_string_buffer(1024)
        for g in range(self.info()["n_groups"]):
            n = C.c_int64()
            check(lib().mcpt_model_group(self.handle, g, buf, 1024, C.byref(n), None))
            a = np.zeros(n.value, np.int32)
            check(lib().mcpt_model_group(self.handle, g, buf, 1024, C.byref(n),
                                         a.ctypes.data_as(C.POINTER(C.c_int32))))
            out[buf.value.decode()] = a
        return out


PIPELINES = {"megakernel": _capi.PIPELINE_MEGAKERNEL, "wavefront": _capi.PIPELINE_WAVEFRONT}
MODES = {"cvmctracer": _capi.MODE_CVMCTRACER, "quinengine": _capi.MODE_QUINENGINE}
GATHERS = {"peer": _capi.GATHER_PEER, "rccl": _capi.GATHER_RCCL}


@dataclass
class RenderParams:
    """Render configuration; defaults are the CVMCTracer constants for scene 1."""
    width: int = IMG_WIDTH
    height: int = IMG_HEIGHT
    spp: int = NUM_SAMPLES_PER_KERNEL
    spp_offset: int = 0
    spp_chunk: int = 32               # summation chunk (part of the result definition)
    max_depth: int = 7                # CUTracer.cu:212
    illum: float = ILLUM
    fov_deg: float = 60.0             # CUTracer.cu:189
    eye: Sequence[float] = (0.0, 5.0, 17.0)
    direction: Sequence[float] = (0.0, 0.0, -1.0)
    up: Sequence[float] = (0.0, 1.0, 0.0)
    seed: int = DEFAULT_SEED
    prev_count: int = 0
    fresnel_kd: bool = True
    tile: int = 8
    shard_count: int = 1
    shard_index: int = 0
    packed: bool = False
    pipeline: str = "megakernel"      # or "wavefront" (C5): identical image, different kernels
    wf_batch: int = 0                 # wavefront paths per batch and stream, 0 = automatic (include/mcpt.h)
    mode: str = "cvmctracer"          # or "quinengine": rtx.hlsl path semantics (see for_quinengine)
    lean: bool = False                # kernels without traversal counters (same image; bench timing)
    wf_sort: bool = False             # wavefront: shade sorts each block of slots by material; same image
    # scheduling (include/mcpt.h): never changes the image or the counters; 0 = automatic
    wf_streams: int = 0               # wavefront HIP streams (1..4)
    wf_refill: int = 0                # wavefront extend: ready lanes before a wave refills
    wf_group_shift: int = 0           # wavefront, global-memory scenes: 2^k paths per segment group
    ready_thresh: int = 0             # megakernel: ready lanes before a shading round
    tail_units_per_lane: int = 0      # megakernel tail split per lane (< 0: off)
    tail_units: int = 0               # megakernel: exact tail-split units (> 0 overrides)
    wf_mem_limit: int = 0             # wavefront queue memory budget in bytes (0: 90% of free)
    force_peer_copy: bool = False     # multi-device: hipMemcpyPeerAsync also between same-device replicas
    gather: str = "peer"              # multi-device shards to devices[0]: "peer" copies or "rccl" (ncclGather)

    @staticmethod
    def for_scene(scene_id: int, **kw) -> "RenderParams":
        """Camera of RenderScene(sceneID) (CUTracer.cu:347-374)."""
        eye = (0.0, 5.0, 17.0) if scene_id == 1 else (0.0, 5.0, 23.0)
        return RenderParams(eye=eye, **kw)

    @staticmethod
    def for_quinengine(**kw) -> "RenderParams":
        """QuinEngine viewer frame (GraphicsRTX.cpp:163-193, rtx.hlsl:373-404): 1 spp,
        depth 5 with Russian roulette, vertical FOV 45, no ILLUM / Fresnel Kd,
        gamma-2.2 running mean; `seed` is the 32-bit frame seed."""
        base = dict(width=640, height=480, spp=1, spp_chunk=1, max_depth=5, illum=1.0, fov_deg=45.0,
                    fresnel_kd=False, seed=0, mode="quinengine")
        base.update(kw)
        return RenderParams(**base)

    def to_c(self) -> RenderParamsC:
        p = RenderParamsC()
        p.width, p.height = int(self.width), int(self.height)
        p.spp, p.spp_offset, p.spp_chunk = int(self.spp), int(self.spp_offset), int(self.spp_chunk)
        p.max_depth, p.illum, p.fov_deg = int(self.max_depth), float(self.illum), float(self.fov_deg)
        p.eye[:] = [float(x) for x in self.eye]
        p.dir[:] = [float(x) for x in self.direction]
        p.up[:] = [float(x) for x in self.up]
        p.seed = int(self.seed) & 0xFFFFFFFFFFFFFFFF
        p.prev_count = int(self.prev_count)
        p.fresnel_kd = 1 if self.fresnel_kd else 0
        p.tile, p.shard_count, p.shard_index = int(self.tile), int(self.shard_count), int(self.shard_index)
        p.packed = 1 if self.packed else 0
        if self.pipeline not in PIPELINES:
            raise ValueError(f"pipeline must be one of {sorted(PIPELINES)}")
        p.pipeline = PIPELINES[self.pipeline]
        p.wf_batch = int(self.wf_batch)
        if self.mode not in MODES:
            raise ValueError(f"mode must be one of {sorted(MODES)}")
        p.mode = MODES[self.mode]
        p.lean = 1 if self.lean else 0
        p.wf_sort = 1 if self.wf_sort else 0
        p.wf_streams, p.wf_refill, p.wf_group_shift = int(self.wf_streams), int(self.wf_refill), int(self.wf_group_shift)
        p.ready_thresh, p.tail_units_per_lane = int(self.ready_thresh), int(self.tail_units_per_lane)
        p.tail_units, p.wf_mem_limit = int(self.tail_units), int(self.wf_mem_limit)
        p.force_peer_copy = 1 if self.force_peer_copy else 0
        if self.gather not in GATHERS:
            raise ValueError(f"gather must be one of {sorted(GATHERS)}")
        p.gather = GATHERS[self.gather]
        return p

    def output_pixels(self) -> int:
        if self.packed or self.shard_count > 1:
            return int(lib().mcpt_shard_pixel_count(C.byref(self.to_c())))
        return int(self.width) * int(self.height)

    def shard_pixels(self) -> np.ndarray:
        """(n, 2) int32 (x, y) of every output slot of a packed/sharded render (-1 = padding)."""
        p = self.to_c()
        n = int(check(lib().mcpt_shard_pixel_count(C.byref(p))))
        xy = np.zeros((n, 2), np.int32)
        check(lib().mcpt_shard_pixels(C.byref(p), xy.ctypes.data_as(C.POINTER(C.c_int32))))
        return xy


class Scene:
    """A device-resident scene (CreateGeometry result + KD tree)."""

    LAYOUTS = {"auto": _capi.LAYOUT_AUTO, "global": _capi.LAYOUT_GLOBAL}
    KD_BUILDS = {"reference": _capi.KD_BUILD_REFERENCE, "sah": _capi.KD_BUILD_SAH}

    def __init__(self, model: ObjModel, host_only: bool = False, kd_cache: Optional[str] = None,
                 layout: str = "auto", kd_build: str = "reference"):
        """kd_cache: directory for the on-disk KD-build cache (mcpt_scene_create_ex);
        ``cache_hit`` tells whether the tree was read from it.  layout "global":
        the scene image with child-box pair records in global memory even if it
        would fit in LDS (MCPT_LAYOUT_GLOBAL).  kd_build "sah": the KD tree's
        splits by the SAH with a traversal cost (MCPT_KD_BUILD_SAH) instead of
        QuinEngine's KDTree.hpp rule -- the same image, fewer node visits."""
        if layout not in self.LAYOUTS:
            raise ValueError(f"layout must be one of {sorted(self.LAYOUTS)}")
        if kd_build not in self.KD_BUILDS:
            raise ValueError(f"kd_build must be one of {sorted(self.KD_BUILDS)}")
        h = C.c_void_p()
        if kd_cache:
            os.makedirs(kd_cache, exist_ok=True)
        opt = _capi.SceneOptions(os.fsencode(kd_cache) if kd_cache else None, int(host_only), self.LAYOUTS[layout],
                                 self.KD_BUILDS[kd_build])
        hit = C.c_int32(0)
        check(lib().mcpt_scene_create_ex(model.handle, C.byref(opt), C.byref(h), C.byref(hit)))
        self.cache_hit = bool(hit.value)
        self._h = h
        self.host_only = host_only

    def close(self):
        h = getattr(self, "_h", None)   # None also when __init__ failed
        if h is not None and _capi._lib is not None:
            _capi._lib.mcpt_scene_destroy(h)
        self._h = None

    __del__ = close

    @property
    def handle(self):
        if self._h is None:
            raise McptError(-1, "scene destroyed")
        return self._h

    def info(self) -> dict:
        i = _capi.SceneInfo()
        check(lib().mcpt_scene_get_info(self.handle, C.byref(i)))
        return {n: int(getattr(i, n)) for n, _ in i._fields_}

    def kd(self):
        """(nodes (n,12) u32, leaf ids, kd_tris, geoms (g,14) f32) as built."""
        i = self.info()
        nodes = np.zeros((i["n_nodes"], 12), np.uint32)
        leafs = np.zeros(max(i["n_leaf_refs"], 1), np.uint32)
        kdt = np.zeros(i["n_triangles"], np.int32)
        geoms = np.zeros((i["n_geometries"], 14), np.float32)
        check(lib().mcpt_scene_copy_kd(self.handle, nodes.ctypes.data_as(C.POINTER(C.c_uint32)),
                                       leafs.ctypes.data_as(C.POINTER(C.c_uint32)),
                                       kdt.ctypes.data_as(C.POINTER(C.c_int32)), _fptr(geoms)))
        return nodes, leafs[: i["n_leaf_refs"]], kdt, geoms

    def render(self, params: RenderParams, fb: Optional[np.ndarray] = None):
        """Synchronous render into a host float32 RGB buffer; returns (fb, stats)."""
        n = params.output_pixels()
        if fb is None:
            fb = np.zeros((n, 3) if (params.packed or params.shard_count > 1) else (params.height, params.width, 3),
                          np.float32)
        if fb.dtype != np.float32 or not fb.flags.c_contiguous or fb.size != 3 * n:
            raise McptError(-1, "fb must be a C-contiguous float32 array with 3 floats per output pixel")
        st = RenderStats()
        check(lib().mcpt_render(self.handle, C.byref(params.to_c()), _fptr(fb), C.byref(st)))
        return fb, st.as_dict()

    def intersect(self, o: np.ndarray, d: np.ndarray, t_max: float = 3.402823466e38):
        """Closest hits of rays (origins o, directions d: (n, 3) float32) on the
        device (CUTracer.cu:44-96 through the render traversal): (kd triangle id
        or -1, (n, 3) beta gamma t, counters)."""
        o = np.ascontiguousarray(o, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
        if o.shape != d.shape:
            raise McptError(-1, "o and d must have the same shape")
        n = o.shape[0]
        tri = np.zeros(n, np.int32)
        hit = np.zeros((n, 3), np.float32)
        st = RenderStats()
        check(lib().mcpt_intersect(self.handle, n, _fptr(o), _fptr(d), C.c_float(t_max),
                                   tri.ctypes.data_as(C.POINTER(C.c_int32)), _fptr(hit), C.byref(st)))
        return tri, hit, st.as_dict()

    def render_unit_counters(self, params: RenderParams):
        """Synchronous render returning (fb, per-unit counters (units, 4): rays, inner, leaf, tests)."""
        n = params.output_pixels()
        fb = np.zeros((n, 3), np.float32)
        chunk = params.spp_chunk if 0 < params.spp_chunk < params.spp else params.spp
        units = n * ((params.spp + chunk - 1) // chunk)
        uc = np.zeros((units, 4), np.uint32)
        check(lib().mcpt_render_unit_counters(self.handle, C.byref(params.to_c()), _fptr(fb),
                                              uc.ctypes.data_as(C.POINTER(C.c_uint32))))
        return fb, uc

    def render_device(self, params: RenderParams, d_fb_rgba_ptr: int, stream_ptr: int = 0):
        """Asynchronous render into a device RGBA float buffer (e.g. a torch tensor's data_ptr())."""
        check(lib().mcpt_render_device(self.handle, C.byref(params.to_c()), C.c_void_p(d_fb_rgba_ptr),
                                       C.c_void_p(stream_ptr)))

    def reserve(self, params: RenderParams):
        check(lib().mcpt_scene_reserve(self.handle, C.byref(params.to_c())))

    def plan(self, params: RenderParams) -> dict:
        """The scheduling a render of `params` would use (streams, batch, thresholds) and
        its device memory (mcpt_plan_query); nothing is allocated or launched."""
        out = _capi.PlanInfo()
        check(lib().mcpt_plan_query(self.handle, C.byref(params.to_c()), C.byref(out)))
        return out.as_dict()

    def stats(self) -> dict:
        st = RenderStats()
        check(lib().mcpt_render_stats_read(self.handle, C.byref(st)))
        return st.as_dict()


class Tracer:
    """PW::Tracer as an object: Initialize / CreateGeometry / DestroyGeometry / RenderScene."""

    def __init__(self):
        self.scene: Optional[Scene] = None
        self.last_stats: dict = {}

    def initialize(self, devices: Sequence[int] = (0,)) -> int:   # CUTracer.cu:220-223 (cudaSetDevice(0))
        """devices[0] holds the scene; more entries replicate scenes created afterwards
        on this thread and split each render into interleaved tiles across them,
        gathered to devices[0] (mcpt_init, include/mcpt.h) -- the same image."""
        arr = (C.c_int32 * len(devices))(*devices)
        return check(lib().mcpt_init(arr, len(devices)))

    def create_geometry(self, model: ObjModel) -> int:             # CUTracer.cu:225-314
        self.destroy_geometry()
        self.scene = Scene(model)
        return 0

    def destroy_geometry(self) -> int:                              # CUTracer.cu:316-338
        if self.scene is not None:
            self.scene.close()
            self.scene = None
        return 0

    def render_scene(self, scene_id: int, hostcolor: np.ndarray, num_kernels: int = NUM_KERNELS,
                     samples_per_kernel: int = NUM_SAMPLES_PER_KERNEL, callback=None, **kw) -> int:
        """RenderScene (CUTracer.cu:340-404): num_kernels launches of samples_per_kernel
        samples; after launch k the buffer holds the running mean (prevCount = k).
        Each launch sums its samples of a pixel in sample order, then divides
        (CUTracer.cu:192-214): spp_chunk 0 unless the caller passes another."""
        if self.scene is None:
            raise McptError(-1, "CreateGeometry has not been called")
        H, W = hostcolor.shape[:2]
        stats = {}
        for each in range(num_kernels):
            kw.setdefault("spp_chunk", 0)
            p = RenderParams.for_scene(scene_id, width=W, height=H, spp=samples_per_kernel,
                                       spp_offset=each * samples_per_kernel, prev_count=each, **kw)
            _, st = self.scene.render(p, hostcolor)
            for k, v in st.items():
                stats[k] = stats.get(k, 0) + v if k != "variant" else v
            if callback is not None:
                callback(each, hostcolor)
        self.last_stats = stats
        return 0

    # reference spellings
    Initialize = initialize
    CreateGeometry = create_geometry
    DestroyGeometry = destroy_geometry
    RenderScene = render_scene


_default = Tracer()


def Initialize() -> int:
    return _default.initialize()


def CreateGeometry(model: ObjModel) -> int:
    return _default.create_geometry(model)


def DestroyGeometry() -> int:
    return _default.destroy_geometry()


def RenderScene(sceneID: int, hostcolor: np.ndarray, **kw) -> int:
    return _default.render_scene(sceneID, hostcolor, **kw)


from .imageio import encode_8bit  # noqa: E402,F401  (main.cpp:19-29 encode; kept here for the API)
