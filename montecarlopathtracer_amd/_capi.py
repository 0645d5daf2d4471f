"""ctypes binding of libmcpt.so (include/mcpt.h).

The library is loaded from this package directory (lib/libmcpt.so, built by
``montecarlopathtracer_amd._build`` / ``__graft_entry__.build()``).  There is
no fallback: if the HIP library is missing or cannot be loaded, importing the
product API raises.  When torch is importable it is imported first so that the
process has a single HIP runtime (torch's libamdhip64.so.7 satisfies the
library's NEEDED entry by soname).
"""
from __future__ import annotations

import ctypes as C
import os

try:  # share torch's HIP runtime when torch is present
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for host-only use
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MCPT_LIB_PATH") or os.path.join(_HERE, "lib", "libmcpt.so")

MCPT_OK = 0
ABI_VERSION = 9
MODE_CVMCTRACER = 0
MODE_QUINENGINE = 1
PIPELINE_MEGAKERNEL = 0
PIPELINE_WAVEFRONT = 1
GATHER_PEER = 0
GATHER_RCCL = 1
ERRORS = {-1: "INVALID", -2: "IO", -3: "PARSE", -4: "DEVICE", -5: "NOMEM", -6: "UNSUPPORTED"}


class McptError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"mcpt error {code} ({ERRORS.get(code, '?')}): {msg}")
        self.code = code


class ModelInfo(C.Structure):
    _fields_ = [(n, C.c_int64) for n in
                ("n_vertices", "n_normals", "n_texcoords", "n_triangles", "n_materials", "n_groups")]


class SceneInfo(C.Structure):
    _fields_ = [(n, C.c_int64) for n in
                ("n_geometries", "n_triangles", "n_nodes", "n_leaf_refs", "kd_depth", "lds_bytes", "device",
                 "node_boxes", "n_devices", "kd_build")]


class RenderParamsC(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32),
        ("spp", C.c_uint32), ("spp_offset", C.c_uint32), ("spp_chunk", C.c_uint32),
        ("max_depth", C.c_int32), ("illum", C.c_float), ("fov_deg", C.c_float),
        ("eye", C.c_float * 3), ("dir", C.c_float * 3), ("up", C.c_float * 3),
        ("seed", C.c_uint64), ("prev_count", C.c_uint32), ("fresnel_kd", C.c_int32),
        ("tile", C.c_int32), ("shard_count", C.c_int32), ("shard_index", C.c_int32), ("packed", C.c_int32),
        ("pipeline", C.c_int32), ("wf_batch", C.c_uint32), ("mode", C.c_int32), ("lean", C.c_int32),
        ("wf_sort", C.c_int32),
        ("wf_streams", C.c_int32), ("wf_refill", C.c_int32), ("wf_group_shift", C.c_int32),
        ("ready_thresh", C.c_int32), ("tail_units_per_lane", C.c_int32), ("tail_units", C.c_int32),
        ("wf_mem_limit", C.c_uint64), ("force_peer_copy", C.c_int32), ("gather", C.c_int32),
    ]


class RenderStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in
                ("rays", "paths", "inner_visits", "leaf_visits", "leaf_refs", "tri_tests", "shades",
                 "stack_spills", "renders")] + [
        ("kernel_ms", C.c_double), ("reduce_ms", C.c_double), ("variant", C.c_int32), ("devices", C.c_int32)]

    def as_dict(self):
        return {n: (getattr(self, n) if isinstance(getattr(self, n), float) else int(getattr(self, n)))
                for n, _ in self._fields_}


class PlanInfo(C.Structure):
    _fields_ = [("pipeline", C.c_int32), ("variant", C.c_int32), ("wf_streams", C.c_int32), ("wf_batch", C.c_uint32),
                ("wf_refill", C.c_int32), ("wf_group_shift", C.c_int32), ("ready_thresh", C.c_int32),
                ("tail_units", C.c_int32), ("work_paths", C.c_uint64), ("workspace_bytes", C.c_uint64), ("wf_queue_bytes", C.c_uint64),
                ("device_free_bytes", C.c_uint64), ("devices", C.c_int32), ("peer_access", C.c_int32),
                ("wf_batch_default", C.c_uint32)]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class SceneOptions(C.Structure):
    _fields_ = [("kd_cache_dir", C.c_char_p), ("host_only", C.c_int32), ("layout", C.c_int32),
                ("kd_build", C.c_int32)]


OBJ_CVMCTRACER = 0
OBJ_TINYOBJ = 1
LAYOUT_AUTO = 0
LAYOUT_GLOBAL = 1
KD_BUILD_REFERENCE = 0
KD_BUILD_SAH = 1


class ModelDesc(C.Structure):
    _fields_ = [
        ("vertices", C.POINTER(C.c_float)), ("n_vertices", C.c_int64),
        ("normals", C.POINTER(C.c_float)), ("n_normals", C.c_int64),
        ("triangles", C.POINTER(C.c_int32)), ("n_triangles", C.c_int64),
        ("materials", C.POINTER(C.c_double)), ("n_materials", C.c_int64),
        ("group_names", C.POINTER(C.c_char_p)), ("group_offsets", C.POINTER(C.c_int64)),
        ("group_tris", C.POINTER(C.c_int32)), ("n_groups", C.c_int64),
    ]


# every symbol include/mcpt.h declares, with its ctypes signature
_vp = C.c_void_p
_SIGS = {
    "mcpt_abi_version": (C.c_int, []),
    "mcpt_last_error": (C.c_char_p, []),
    "mcpt_init": (C.c_int, [C.POINTER(C.c_int32), C.c_int32]),
    "mcpt_device_count": (C.c_int, [C.POINTER(C.c_int32)]),
    "mcpt_render_params_default": (None, [C.POINTER(RenderParamsC)]),
    "mcpt_render_params_quinengine": (None, [C.POINTER(RenderParamsC)]),
    "mcpt_model_create": (C.c_int, [C.POINTER(ModelDesc), C.POINTER(_vp)]),
    "mcpt_model_read_obj": (C.c_int, [C.c_char_p, C.POINTER(_vp)]),
    "mcpt_model_read_obj_ex": (C.c_int, [C.c_char_p, C.c_int32, C.POINTER(_vp)]),
    "mcpt_model_free": (None, [_vp]),
    "mcpt_model_get_info": (C.c_int, [_vp, C.POINTER(ModelInfo)]),
    "mcpt_model_copy_vertices": (C.c_int, [_vp, C.POINTER(C.c_float)]),
    "mcpt_model_copy_normals": (C.c_int, [_vp, C.POINTER(C.c_float)]),
    "mcpt_model_copy_triangles": (C.c_int, [_vp, C.POINTER(C.c_int32)]),
    "mcpt_model_copy_materials": (C.c_int, [_vp, C.POINTER(C.c_double)]),
    "mcpt_model_group": (C.c_int, [_vp, C.c_int64, C.c_char_p, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
    "mcpt_scene_create": (C.c_int, [_vp, C.POINTER(_vp)]),
    "mcpt_scene_create_host": (C.c_int, [_vp, C.POINTER(_vp)]),
    "mcpt_scene_create_cached": (C.c_int, [_vp, C.c_char_p, C.c_int32, C.POINTER(_vp), C.POINTER(C.c_int32)]),
    "mcpt_scene_create_ex": (C.c_int, [_vp, C.POINTER(SceneOptions), C.POINTER(_vp), C.POINTER(C.c_int32)]),
    "mcpt_scene_destroy": (None, [_vp]),
    "mcpt_scene_get_info": (C.c_int, [_vp, C.POINTER(SceneInfo)]),
    "mcpt_scene_copy_kd": (C.c_int, [_vp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_int32),
                                     C.POINTER(C.c_float)]),
    "mcpt_render": (C.c_int, [_vp, C.POINTER(RenderParamsC), C.POINTER(C.c_float), C.POINTER(RenderStats)]),
    "mcpt_render_device": (C.c_int, [_vp, C.POINTER(RenderParamsC), _vp, _vp]),
    "mcpt_render_unit_counters": (C.c_int, [_vp, C.POINTER(RenderParamsC), C.POINTER(C.c_float),
                                            C.POINTER(C.c_uint32)]),
    "mcpt_render_stats_read": (C.c_int, [_vp, C.POINTER(RenderStats)]),
    "mcpt_intersect": (C.c_int, [_vp, C.c_int64, C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_float,
                                 C.POINTER(C.c_int32), C.POINTER(C.c_float), C.POINTER(RenderStats)]),
    "mcpt_shard_pixel_count": (C.c_int64, [C.POINTER(RenderParamsC)]),
    "mcpt_shard_pixels": (C.c_int, [C.POINTER(RenderParamsC), C.POINTER(C.c_int32)]),
    "mcpt_scene_reserve": (C.c_int, [_vp, C.POINTER(RenderParamsC)]),
    "mcpt_plan_query": (C.c_int, [_vp, C.POINTER(RenderParamsC), C.POINTER(PlanInfo)]),
}

_lib = None


def lib():
    """Load libmcpt.so (raises if it was not built -- no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; "
                              f"g.build()'` or `python -m montecarlopathtracer_amd._build`")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.mcpt_abi_version() != ABI_VERSION:
            raise ImportError("libmcpt.so ABI version mismatch")
        _lib = L
    return _lib


def check(rc: int) -> int:
    if rc < 0:
        raise McptError(rc, lib().mcpt_last_error().decode(errors="replace"))
    return rc


def declared_symbols():
    return list(_SIGS)
