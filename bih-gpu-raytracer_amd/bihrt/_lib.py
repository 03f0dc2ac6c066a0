"""ctypes binding of libbih_amd.so (include/bih.h).

The library is built in-tree (`make -C bih-gpu-raytracer_amd`, or
__graft_entry__.build()).  There is no CPU fallback: if the shared object is
missing, loading raises, and every render/build call needs a HIP device.
"""
from __future__ import annotations

import ctypes as C
import os
import re

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.environ.get("BIH_LIB") or os.path.join(PKG_DIR, "lib", "libbih_amd.so")
HEADER_PATH = os.path.join(REPO_DIR, "include", "bih.h")

BIH_OK = 0
ERRORS = {
    -1: "BIH_ERR_INVALID", -2: "BIH_ERR_NO_DEVICE", -3: "BIH_ERR_HIP", -4: "BIH_ERR_OOM",
    -5: "BIH_ERR_NONFINITE", -6: "BIH_ERR_TOO_LARGE", -7: "BIH_ERR_MISMATCH",
    -8: "BIH_ERR_IO", -9: "BIH_ERR_PARSE",
}
TRAVERSE_ANYHIT, TRAVERSE_REFERENCE = 0, 1
PARAM_ITEM_TILES, PARAM_PAIR_CAP, PARAM_BINS_CAP, PARAM_FORCE_FALLBACK, PARAM_WHITTED_COUNTERS = 1, 2, 3, 4, 5   # bih_tree_set_param
PARAM_STATIC_SOUP = 6
PARAM_TEST_ALLOC_FAIL = 7   # tests: the next allocating build fails at its k-th allocation
(ARR_MORTON_SORTED, ARR_TRI_INDEX, ARR_UNIQUE_MC, ARR_DUP_COUNT, ARR_FIRST_IDX, ARR_LEAF_PARENT,
 ARR_CLIP, ARR_AXIS, ARR_CHILDREN, ARR_IS_LEAF, ARR_PARENT, ARR_TRI_LO, ARR_TRI_HI) = range(13)


class BihError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        name = ERRORS.get(code, str(code))
        msg = strerror(code) if _lib is not None else name
        super().__init__(f"{what}: {name} ({msg})" if what else f"{name} ({msg})")


class Scene(C.Structure):
    _fields_ = [("n_tris", C.c_uint32), ("v", C.c_void_p)]


class Camera(C.Structure):
    _fields_ = [("origin", C.c_float * 3), ("lower_left", C.c_float * 3),
                ("horizontal", C.c_float * 3), ("vertical", C.c_float * 3)]

    def as_list(self):
        return list(self.origin) + list(self.lower_left) + list(self.horizontal) + list(self.vertical)

    @classmethod
    def from_list(cls, v):
        c = cls()
        v = [float(x) for x in v]
        for i in range(3):
            c.origin[i], c.lower_left[i] = v[i], v[3 + i]
            c.horizontal[i], c.vertical[i] = v[6 + i], v[9 + i]
        return c


class Framebuffer(C.Structure):
    _fields_ = [("w", C.c_uint32), ("h", C.c_uint32), ("spp", C.c_uint32), ("frame", C.c_uint32),
                ("seed", C.c_uint64), ("rgba", C.c_void_p)]


class Rows(C.Structure):
    _fields_ = [("row0", C.c_uint32), ("nrows", C.c_uint32), ("band_h", C.c_uint32),
                ("band_step", C.c_uint32)]


class BinsStats(C.Structure):
    _fields_ = [("usable", C.c_uint32), ("tiles_x", C.c_uint32), ("tiles_y", C.c_uint32),
                ("list_entries", C.c_uint64), ("global_entries", C.c_uint32)]


class TreeInfo(C.Structure):
    _fields_ = [("n_tris", C.c_uint32), ("n_unique", C.c_uint32), ("scene_lo", C.c_float * 3),
                ("scene_hi", C.c_float * 3), ("device", C.c_int), ("device_bytes", C.c_uint64),
                ("build_ms", C.c_double), ("device_allocs", C.c_uint64)]


_lib = None


def exported_symbols_from_header(path: str = HEADER_PATH):
    """Function names declared in include/bih.h."""
    src = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w[\w\s\*]*?\b(bih_\w+)\s*\(", src, re.M)))


def load():
    """Loads the in-tree shared object (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(f"{LIB_PATH} not built: run `make -C bih-gpu-raytracer_amd` "
                      "(or __graft_entry__.build())")
    # One HIP runtime per process: the torch wheel bundles its own
    # libamdhip64 (soname libamdhip64.so.7, NEEDED as "libamdhip64.so"), so
    # if torch is present it is loaded first and libbih_amd.so binds to that
    # same runtime instead of pulling in a second copy from /opt/rocm.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
    L.bih_abi_version.restype = i32
    L.bih_device_count.restype = i32
    L.bih_strerror.argtypes = [i32]
    L.bih_strerror.restype = C.c_char_p
    L.bih_camera_reference.argtypes = [u32, u32, C.POINTER(Camera)]
    L.bih_camera_ray_bound.argtypes = [C.POINTER(Camera), C.POINTER(C.c_float)]
    L.bih_scene_load_obj.argtypes = [C.c_char_p, C.POINTER(Scene), C.POINTER(u32)]
    L.bih_scene_free.argtypes = [C.POINTER(Scene)]
    L.bih_scene_free.restype = None
    L.bih_build.argtypes = [C.POINTER(Scene), i32, C.POINTER(vp)]
    L.bih_build_device.argtypes = [vp, u32, i32, vp, C.POINTER(vp)]
    L.bih_rebuild.argtypes = [vp]
    L.bih_free.argtypes = [vp]
    L.bih_free.restype = None
    L.bih_tree_get_info.argtypes = [vp, C.POINTER(TreeInfo)]
    L.bih_tree_export.argtypes = [vp, i32, vp, C.POINTER(C.c_size_t)]
    L.bih_render.argtypes = [C.POINTER(Scene), vp, C.POINTER(Camera), C.POINTER(Framebuffer)]
    L.bih_render_rows.argtypes = [C.POINTER(Scene), vp, C.POINTER(Camera), C.POINTER(Framebuffer),
                                  u32, u32]
    L.bih_render_device.argtypes = [vp, C.POINTER(Camera), u32, u32, u32, u32, u64,
                                    C.POINTER(Rows), u32, vp, vp, vp]
    L.bih_sync.argtypes = [vp, vp]
    L.bih_render_device_frames.argtypes = [vp, C.POINTER(Camera), u32, u32, u32, u32, u32, u64,
                                           C.POINTER(Rows), vp, u64, vp]
    L.bih_render_whitted_device.argtypes = [vp, C.POINTER(Camera), u32, u32, u32, u32, u64,
                                            C.POINTER(Rows), vp, vp, vp]
    L.bih_render_whitted.argtypes = [C.POINTER(Scene), vp, C.POINTER(Camera), C.POINTER(Framebuffer)]
    L.bih_last_render_ms.argtypes = [vp, C.POINTER(C.c_double)]
    L.bih_set_timing.argtypes = [vp, i32]
    L.bih_last_render_times.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.bih_bins_get_stats.argtypes = [vp, C.POINTER(BinsStats)]
    L.bih_reserve.argtypes = [vp, u32, u32, u32, C.POINTER(Rows), u32]
    L.bih_tree_set_param.argtypes = [vp, i32, u64]
    L.bih_whitted_work.argtypes = [vp, C.POINTER(u32), C.POINTER(u64), C.POINTER(u64)]
    L.bih_host_register.argtypes = [vp, C.c_size_t]
    L.bih_host_unregister.argtypes = [vp]
    L.bih_render_history.argtypes = [vp, u32, C.POINTER(C.c_double)]
    for name in ("bih_camera_reference", "bih_camera_ray_bound", "bih_scene_load_obj", "bih_build", "bih_build_device", "bih_rebuild",
                 "bih_tree_get_info", "bih_tree_export", "bih_render", "bih_render_rows",
                 "bih_render_device", "bih_sync", "bih_last_render_ms", "bih_last_render_times", "bih_set_timing",
                 "bih_render_whitted_device", "bih_render_whitted", "bih_render_device_frames",
                 "bih_bins_get_stats", "bih_reserve", "bih_tree_set_param", "bih_whitted_work",
                 "bih_host_register", "bih_host_unregister", "bih_render_history"):
        getattr(L, name).restype = i32
    _lib = L
    return L


def strerror(code: int) -> str:
    return load().bih_strerror(code).decode()


def check(rc: int, what: str = ""):
    if rc != BIH_OK:
        raise BihError(rc, what)
    return rc
