"""ctypes binding of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module.  It is the checker, never the thing measured or shipped.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "lib", "libbih_oracle.so")

MODE_GPU_REF, MODE_BRUTE, MODE_HOST_DEBUG, MODE_GPU_ANYHIT = 0, 1, 2, 3


class _Tree(C.Structure):
    _fields_ = [
        ("n_tris", C.c_int32), ("n_unique", C.c_int32),
        ("scene_lo", C.c_float * 3), ("scene_hi", C.c_float * 3),
        ("lo", C.POINTER(C.c_float)), ("hi", C.POINTER(C.c_float)),
        ("center", C.POINTER(C.c_float)), ("norm", C.POINTER(C.c_float)),
        ("morton", C.POINTER(C.c_uint32)), ("tri_idx", C.POINTER(C.c_uint32)),
        ("unique_mc", C.POINTER(C.c_uint32)), ("dup_cnt", C.POINTER(C.c_uint32)),
        ("first_idx", C.POINTER(C.c_int32)), ("leaf_parent", C.POINTER(C.c_int32)),
        ("clip", C.POINTER(C.c_float)), ("axis", C.POINTER(C.c_int32)),
        ("children", C.POINTER(C.c_int32)), ("is_leaf", C.POINTER(C.c_uint8)),
        ("parent", C.POINTER(C.c_int32)), ("tris", C.POINTER(C.c_float)),
    ]


class Stats(C.Structure):
    _fields_ = [
        ("rays", C.c_uint64), ("rays_hit", C.c_uint64), ("node_visits", C.c_uint64),
        ("leaf_visits", C.c_uint64), ("tri_tests", C.c_uint64), ("slab_miss", C.c_uint64),
        ("max_stack", C.c_int32), ("threads", C.c_int32), ("render_seconds", C.c_double),
        ("push_at", C.c_uint64 * 33),
    ]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["push_at"] = list(self.push_at)
        return d


_lib = None


def build_lib() -> str:
    """Compile the oracle with its committed Makefile (gcc, strict IEEE)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build_lib()
        L = C.CDLL(LIB)
        L.ob_build.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.POINTER(_Tree))]
        L.ob_build.restype = C.c_int
        L.ob_free.argtypes = [C.POINTER(_Tree)]
        L.ob_camera_reference.argtypes = [C.c_uint32, C.c_uint32, C.c_void_p]
        L.ob_rng_state.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p]
        L.ob_rng_uniform.argtypes = [C.c_void_p, C.c_void_p]
        L.ob_rng_uniform.restype = C.c_float
        L.ob_rng_next.argtypes = [C.c_void_p, C.c_void_p]
        L.ob_rng_next.restype = C.c_uint32
        L.ob_render.argtypes = [C.POINTER(_Tree), C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32,
                                C.c_void_p, C.c_int, C.c_int, C.POINTER(Stats), C.c_void_p]
        L.ob_render.restype = C.c_int
        L.ob_trace_rays.argtypes = [C.POINTER(_Tree), C.c_void_p, C.c_void_p, C.c_int32, C.c_int,
                                    C.c_void_p, C.c_void_p, C.c_void_p]
        L.ob_trace_rays.restype = C.c_int
        L.ob_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.ob_mt.restype = C.c_int
        L.ob_render_whitted.argtypes = [C.POINTER(_Tree), C.c_void_p, C.c_uint32, C.c_uint32,
                                        C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32,
                                        C.c_uint32, C.c_void_p, C.c_int, C.POINTER(Stats),
                                        C.c_void_p]
        L.ob_render_whitted.restype = C.c_int
        L.ob_closest.argtypes = [C.POINTER(_Tree), C.c_void_p, C.c_void_p, C.c_float, C.c_void_p,
                                 C.c_void_p]
        L.ob_closest.restype = C.c_int
        L.ob_morton3d.argtypes = [C.c_float, C.c_float, C.c_float]
        L.ob_morton3d.restype = C.c_uint32
        _lib = L
    return _lib


def _arr(ptr, n, dtype):
    if n <= 0:
        return np.zeros(0, dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


class OracleTree:
    """Oracle BIH for a float32 (n,9) soup; arrays mirror GPUArrayManager."""

    def __init__(self, tris: np.ndarray):
        tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
        self.tris = tris
        p = C.POINTER(_Tree)()
        rc = lib().ob_build(tris.ctypes.data, tris.shape[0], C.byref(p))
        if rc != 0:
            raise RuntimeError(f"ob_build failed: {rc}")
        self._p = p
        t = p.contents
        n, U = t.n_tris, t.n_unique
        m = max(U - 1, 0)
        self.n, self.U = n, U
        self.scene_lo = np.array(t.scene_lo[:], np.float32)
        self.scene_hi = np.array(t.scene_hi[:], np.float32)
        self.lo = _arr(t.lo, 3 * n, np.float32).reshape(-1, 3)
        self.hi = _arr(t.hi, 3 * n, np.float32).reshape(-1, 3)
        self.center = _arr(t.center, 3 * n, np.float32).reshape(-1, 3)
        self.norm = _arr(t.norm, 3 * n, np.float32).reshape(-1, 3)
        self.morton = _arr(t.morton, n, np.uint32)
        self.tri_idx = _arr(t.tri_idx, n, np.uint32)
        self.unique_mc = _arr(t.unique_mc, U, np.uint32)
        self.dup_cnt = _arr(t.dup_cnt, U, np.uint32)
        self.first_idx = _arr(t.first_idx, U, np.int32)
        self.leaf_parent = _arr(t.leaf_parent, U, np.int32)
        self.clip = _arr(t.clip, 2 * m, np.float32).reshape(-1, 2)
        self.axis = _arr(t.axis, m, np.int32)
        self.children = _arr(t.children, 2 * m, np.int32).reshape(-1, 2)
        self.is_leaf = _arr(t.is_leaf, 2 * m, np.uint8).reshape(-1, 2)
        self.parent = _arr(t.parent, m, np.int32)

    def __del__(self):
        try:
            lib().ob_free(self._p)
        except Exception:
            pass

    def render(self, w, h, spp=4, frame=0, seed=1984, cam=None, rows=None, mode=MODE_GPU_REF,
               threads=0, ray_stats=False):
        """Returns (uint32 image rows, Stats[, (rays, 3) u32 {nodes, leaves, tris}]).
        rows = (row0, nrows, step)."""
        if cam is None:
            cam = camera_reference(w, h)
        cam = np.ascontiguousarray(cam, np.float32).reshape(12)
        row0, nrows, step = rows if rows is not None else (0, h, 1)
        out = np.zeros((nrows, w), np.uint32)
        st = Stats()
        rc_arr = np.zeros((nrows * w * spp, 3), np.uint32) if ray_stats else None
        rc = lib().ob_render(self._p, cam.ctypes.data, w, h, spp, frame, seed, row0, nrows, step,
                             out.ctypes.data, mode, threads, C.byref(st),
                             rc_arr.ctypes.data if ray_stats else None)
        if rc != 0:
            raise RuntimeError(f"ob_render failed: {rc}")
        if ray_stats:
            return out, st, rc_arr
        return out, st

    def render_whitted(self, w, h, spp=4, frame=0, seed=1984, cam=None, rows=None, threads=0,
                       depths=False):
        """Config C4 (bih_oracle.h ob_render_whitted): (uint32 image rows, Stats[,
        uint8 per-sample hit counts (rays, )]).  Stats.slab_miss = rays traced."""
        if cam is None:
            cam = camera_reference(w, h)
        cam = np.ascontiguousarray(cam, np.float32).reshape(12)
        row0, nrows, step = rows if rows is not None else (0, h, 1)
        out = np.zeros((nrows, w), np.uint32)
        st = Stats()
        dep = np.zeros(nrows * w * spp, np.uint8) if depths else None
        rc = lib().ob_render_whitted(self._p, cam.ctypes.data, w, h, spp, frame, seed, row0, nrows,
                                     step, out.ctypes.data, threads, C.byref(st),
                                     dep.ctypes.data if depths else None)
        if rc != 0:
            raise RuntimeError(f"ob_render_whitted failed: {rc}")
        return (out, st, dep) if depths else (out, st)

    def closest(self, o, d, t_lo=0.0):
        """C4 closest hit: (t, sorted index) or (FLT_MAX, -1)."""
        o = np.ascontiguousarray(o, np.float32).reshape(3)
        d = np.ascontiguousarray(d, np.float32).reshape(3)
        t = np.zeros(1, np.float32)
        i = np.zeros(1, np.int32)
        lib().ob_closest(self._p, o.ctypes.data, d.ctypes.data, t_lo, t.ctypes.data, i.ctypes.data)
        return float(t[0]), int(i[0])

    def trace(self, orig, dirs, mode=MODE_GPU_REF):
        orig = np.ascontiguousarray(orig, np.float32).reshape(-1, 3)
        dirs = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
        n = orig.shape[0]
        hit = np.zeros(n, np.uint8)
        nodes = np.zeros(n, np.uint32)
        tris = np.zeros(n, np.uint32)
        lib().ob_trace_rays(self._p, orig.ctypes.data, dirs.ctypes.data, n, mode, hit.ctypes.data,
                            nodes.ctypes.data, tris.ctypes.data)
        return hit, nodes, tris


def camera_reference(w: int, h: int) -> np.ndarray:
    cam = np.zeros(12, np.float32)
    lib().ob_camera_reference(w, h, cam.ctypes.data)
    return cam


def rng_state(seed: int, subseq: int, skip: int = 0):
    v = np.zeros(5, np.uint32)
    d = np.zeros(1, np.uint32)
    lib().ob_rng_state(seed, subseq, skip, v.ctypes.data, d.ctypes.data)
    return v, d


def rng_uniforms(seed: int, subseq: int, count: int, skip: int = 0) -> np.ndarray:
    v, d = rng_state(seed, subseq, skip)
    return np.array([lib().ob_rng_uniform(v.ctypes.data, d.ctypes.data) for _ in range(count)],
                    np.float32)


def mt(tri, o, d):
    tri = np.ascontiguousarray(tri, np.float32).reshape(9)
    o = np.ascontiguousarray(o, np.float32).reshape(3)
    d = np.ascontiguousarray(d, np.float32).reshape(3)
    t = np.zeros(1, np.float32)
    r = lib().ob_mt(tri.ctypes.data, o.ctypes.data, d.ctypes.data, t.ctypes.data)
    return bool(r), float(t[0])


def morton3d(x, y, z) -> int:
    return int(lib().ob_morton3d(x, y, z))
