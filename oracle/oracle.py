"""ctypes binding of the CPU oracle (oracle/build/libmcpt_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker / CPU reference timing.  The
product package never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libmcpt_oracle.so")

BRUTE, KD_REF, KD_ORDERED = 0, 1, 2
MODE_CV, MODE_QE = 0, 1


class Params(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32),
        ("x0", C.c_int32), ("y0", C.c_int32), ("x1", C.c_int32), ("y1", C.c_int32),
        ("spp", C.c_uint32), ("spp_offset", C.c_uint32), ("spp_chunk", C.c_uint32),
        ("max_depth", C.c_int32), ("illum", C.c_float), ("tan_half_fov", C.c_float),
        ("eye", C.c_float * 3), ("fwd", C.c_float * 3), ("up", C.c_float * 3), ("right", C.c_float * 3),
        ("seed", C.c_uint64), ("traversal", C.c_int32), ("threads", C.c_int32),
        ("prev_count", C.c_uint32), ("fresnel_kd", C.c_int32),
        ("mode", C.c_int32), ("proj11", C.c_float), ("proj22", C.c_float), ("node_boxes", C.c_int32),
    ]


class Counters(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in
                ("rays", "paths", "inner_visits", "leaf_visits", "leaf_refs", "tri_tests", "shades", "stack_max")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


def build() -> str:
    """Compile the oracle with its Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, f32p, i32p, u32p = C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_int32), C.POINTER(C.c_uint32)
        L.orc_scene_load.restype = vp
        L.orc_scene_load.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
        L.orc_scene_load_ex.restype = vp
        L.orc_scene_load_ex.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_int]
        L.orc_scene_load_kd.restype = vp
        L.orc_scene_load_kd.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_char_p, C.c_int]
        L.orc_kd_set_sah_costs.argtypes = [C.c_float, C.c_float]
        L.orc_scene_free.argtypes = [vp]
        L.orc_scene_info.argtypes = [vp, C.POINTER(C.c_int64)]
        for n in ("orc_copy_vertices", "orc_copy_normals"):
            getattr(L, n).argtypes = [vp, f32p]
        L.orc_copy_triangles.argtypes = [vp, i32p]
        L.orc_copy_materials.argtypes = [vp, C.POINTER(C.c_double)]
        L.orc_group_name.restype = C.c_char_p
        L.orc_group_name.argtypes = [vp, C.c_int]
        L.orc_group_ntris.argtypes = [vp, C.c_int]
        L.orc_group_tris.argtypes = [vp, C.c_int, i32p]
        L.orc_copy_geoms.argtypes = [vp, f32p]
        L.orc_copy_kd_tris.argtypes = [vp, i32p]
        L.orc_copy_kd_nodes.argtypes = [vp, u32p]
        L.orc_copy_kd_leaf_ids.argtypes = [vp, u32p]
        L.orc_det3.restype = C.c_float
        L.orc_det3.argtypes = [f32p]
        L.orc_tea16.restype = C.c_uint32
        L.orc_tea16.argtypes = [C.c_uint32, C.c_uint32]
        L.orc_pcg_hash.restype = C.c_uint32
        L.orc_pcg_hash.argtypes = [C.c_uint32]
        L.orc_rng_init.restype = C.c_uint32
        L.orc_rng_init.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
        L.orc_rng_next.restype = C.c_float
        L.orc_rng_next.argtypes = [u32p]
        L.orc_seed_key.restype = C.c_uint32
        L.orc_seed_key.argtypes = [C.c_uint64]
        for n in ("orc_sinf", "orc_cosf"):
            getattr(L, n).restype = C.c_float
            getattr(L, n).argtypes = [C.c_float]
        L.orc_powf.restype = C.c_float
        L.orc_powf.argtypes = [C.c_float, C.c_float]
        L.orc_pow5f.restype = C.c_float
        L.orc_pow5f.argtypes = [C.c_float]
        L.orc_sample_hemi.argtypes = [f32p, f32p, f32p]
        L.orc_sample_phong.argtypes = [f32p, f32p, C.c_uint32, f32p, f32p]
        L.orc_sample_fresnel.argtypes = [f32p, f32p, C.c_float, C.c_float, f32p, f32p]
        L.orc_sample_phong_qe.argtypes = [f32p, f32p, C.c_float, f32p, f32p]
        L.orc_sample_fresnel_qe.argtypes = [f32p, f32p, C.c_float, C.c_float, f32p, f32p]
        L.orc_tan_half_fov.restype = C.c_float
        L.orc_tan_half_fov.argtypes = [C.c_float]
        L.orc_qe_proj.restype = None
        L.orc_qe_proj.argtypes = [C.c_float, C.c_int32, C.c_int32, f32p, f32p]
        L.orc_camera_basis.argtypes = [f32p] * 6
        L.orc_intersect_batch.argtypes = [vp, C.c_int, C.c_int64, f32p, f32p, i32p, i32p, f32p, C.POINTER(Counters)]
        L.orc_intersect_batch_mt.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int64, f32p, f32p, i32p, i32p, f32p,
                                             C.POINTER(Counters)]
        L.orc_render.restype = C.c_int
        L.orc_render.argtypes = [vp, C.POINTER(Params), f32p, C.POINTER(Counters)]
        _lib = L
    return _lib


def _p(a, ct):
    return a.ctypes.data_as(C.POINTER(ct))


class Scene:
    """An oracle scene (model + CreateGeometry groups + reference KD tree)."""

    KD_BUILDS = {"reference": 0, "sah": 1}

    def __init__(self, obj_path: str, flavor: str = "cvmctracer", kd_build: str = "reference"):
        """flavor "tinyobj": QuinEngine's loader semantics (obj_reader.c orc_model_read_tinyobj);
        kd_build "sah": the product's MCPT_KD_BUILD_SAH split rule (kdtree_ref.c sah_split)"""
        L = lib()
        err = C.create_string_buffer(512)
        h = L.orc_scene_load_kd(obj_path.encode(), {"cvmctracer": 0, "tinyobj": 1}[flavor], self.KD_BUILDS[kd_build],
                                err, 512)
        if not h:
            raise RuntimeError(f"oracle: {err.value.decode()}")
        self._h = h
        info = np.zeros(10, np.int64)
        L.orc_scene_info(h, _p(info, C.c_int64))
        (self.nverts, self.nnormals, self.ntris, self.nmats, self.ngroups, self.ngeoms,
         self.nkd, self.nnodes, self.nleaf_ids, self.kd_depth) = [int(v) for v in info]

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.orc_scene_free(h)
            self._h = None

    # --- dumps ------------------------------------------------------------
    def vertices(self):
        a = np.zeros((self.nverts, 3), np.float32); lib().orc_copy_vertices(self._h, _p(a, C.c_float)); return a

    def normals(self):
        a = np.zeros((self.nnormals, 3), np.float32); lib().orc_copy_normals(self._h, _p(a, C.c_float)); return a

    def triangles(self):
        a = np.zeros((self.ntris, 10), np.int32); lib().orc_copy_triangles(self._h, _p(a, C.c_int32)); return a

    def materials(self):
        a = np.zeros((self.nmats, 12), np.float64); lib().orc_copy_materials(self._h, _p(a, C.c_double)); return a

    def groups(self):
        out = {}
        for g in range(self.ngroups):
            n = lib().orc_group_ntris(self._h, g)
            a = np.zeros(n, np.int32)
            if n:
                lib().orc_group_tris(self._h, g, _p(a, C.c_int32))
            out[lib().orc_group_name(self._h, g).decode()] = a
        return out

    def geoms(self):
        a = np.zeros((self.ngeoms, 14), np.float32); lib().orc_copy_geoms(self._h, _p(a, C.c_float)); return a

    def kd_tris(self):
        a = np.zeros(self.nkd, np.int32); lib().orc_copy_kd_tris(self._h, _p(a, C.c_int32)); return a

    def kd_nodes(self):
        a = np.zeros((self.nnodes, 12), np.uint32); lib().orc_copy_kd_nodes(self._h, _p(a, C.c_uint32)); return a

    def kd_verts(self):
        """(n_kd, 3, 3) float32 vertex positions of the KD triangles (kd id order)"""
        v, t = self.vertices(), self.triangles()
        return v[t[self.kd_tris()][:, :3]].astype(np.float32)

    def kd_leaf_ids(self):
        a = np.zeros(max(self.nleaf_ids, 1), np.uint32); lib().orc_copy_kd_leaf_ids(self._h, _p(a, C.c_uint32))
        return a[: self.nleaf_ids]

    # --- queries ----------------------------------------------------------
    def intersect(self, o, d, traversal=BRUTE, node_boxes=0, threads=1):
        """closest hits: (kd triangle id or -1, geometry, (beta, gamma, t, hit point) x6 floats, counters)"""
        o = np.ascontiguousarray(o, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
        n = o.shape[0]
        tri = np.zeros(n, np.int32); geom = np.zeros(n, np.int32); hit = np.zeros((n, 6), np.float32)
        c = Counters()
        lib().orc_intersect_batch_mt(self._h, traversal, node_boxes, threads, n, _p(o, C.c_float), _p(d, C.c_float),
                                     _p(tri, C.c_int32), _p(geom, C.c_int32), _p(hit, C.c_float), C.byref(c))
        return tri, geom, hit, c.as_dict()

    def render(self, params: "RenderParams", out=None):
        W, H = params.width, params.height
        if out is None:
            out = np.zeros((H, W, 3), np.float32)
        P = params.to_c()
        c = Counters()
        rc = lib().orc_render(self._h, C.byref(P), _p(out, C.c_float), C.byref(c))
        if rc != 0:
            raise RuntimeError("oracle render failed")
        return out, c.as_dict()


def camera_basis(eye, direction, up):
    L = lib()
    f = np.zeros(3, np.float32); u = np.zeros(3, np.float32); r = np.zeros(3, np.float32)
    e = np.asarray(eye, np.float32); d = np.asarray(direction, np.float32); up_ = np.asarray(up, np.float32)
    L.orc_camera_basis(_p(e, C.c_float), _p(d, C.c_float), _p(up_, C.c_float),
                       _p(f, C.c_float), _p(u, C.c_float), _p(r, C.c_float))
    return f, u, r


class RenderParams:
    """Same fields/defaults as montecarlopathtracer_amd.RenderParams (CVMCTracer constants)."""

    def __init__(self, width=64, height=64, spp=4, spp_offset=0, spp_chunk=0, max_depth=7, illum=10.0,
                 fov=60.0, scene_id=1, eye=None, direction=(0, 0, -1), up=(0, 1, 0), seed=0x4D435054,
                 traversal=KD_ORDERED, threads=1, region=None, prev_count=0, fresnel_kd=1, mode=MODE_CV,
                 node_boxes=0):
        self.width, self.height, self.spp, self.spp_offset, self.spp_chunk = width, height, spp, spp_offset, spp_chunk
        self.max_depth, self.illum, self.fov, self.seed = max_depth, illum, fov, seed
        if eye is None:
            eye = (0.0, 5.0, 17.0) if scene_id == 1 else (0.0, 5.0, 23.0)   # CUTracer.cu:349,363
        self.eye, self.direction, self.up = eye, direction, up
        self.traversal, self.threads, self.prev_count, self.fresnel_kd = traversal, threads, prev_count, fresnel_kd
        self.region = region or (0, 0, width, height)
        self.mode = mode
        self.node_boxes = node_boxes

    def to_c(self):
        P = Params()
        P.width, P.height = self.width, self.height
        P.x0, P.y0, P.x1, P.y1 = self.region
        P.spp, P.spp_offset, P.spp_chunk = self.spp, self.spp_offset, self.spp_chunk
        P.max_depth, P.illum = self.max_depth, self.illum
        P.tan_half_fov = lib().orc_tan_half_fov(self.fov)
        f, u, r = camera_basis(self.eye, self.direction, self.up)
        P.eye[:] = [float(x) for x in self.eye]
        P.fwd[:] = f.tolist(); P.up[:] = u.tolist(); P.right[:] = r.tolist()
        P.seed = self.seed
        P.traversal, P.threads, P.prev_count, P.fresnel_kd = self.traversal, self.threads, self.prev_count, self.fresnel_kd
        P.mode = self.mode
        P.node_boxes = self.node_boxes
        if self.mode == MODE_QE:
            p11, p22 = C.c_float(), C.c_float()
            lib().orc_qe_proj(C.c_float(self.fov), self.width, self.height, C.byref(p11), C.byref(p22))
            P.proj11, P.proj22 = p11.value, p22.value
        return P
