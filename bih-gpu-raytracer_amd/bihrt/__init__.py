"""bihrt -- Python host side of the MI355X BIH ray tracer.

Mirrors the reference's host interface for the hot path
(rehakvoj1/BIH-GPU-Raytracer, BIH_Raytracer/BIH_Raytracer/src):

  GPUArrayManager  (GPUArrayManager.h:6-56)  -> bihrt.GPUArrayManager: owns the
                   scene soup and the BIH on one device (bih_build/bih_rebuild)
  Renderer.Init / Render / Launch_cudaRender (Renderer.h:18-27) ->
                   bihrt.Renderer: camera, framebuffer, persistent RNG state,
                   render(g_odata) per frame

Everything runs through libbih_amd.so (HIP, gfx950); there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import scenes  # noqa: F401
from ._lib import (PARAM_BINS_CAP, PARAM_FORCE_FALLBACK, PARAM_ITEM_TILES, PARAM_PAIR_CAP, PARAM_STATIC_SOUP,
                   PARAM_TEST_ALLOC_FAIL, PARAM_WHITTED_COUNTERS,
                   TRAVERSE_ANYHIT,
                   TRAVERSE_REFERENCE, BihError, Camera, Framebuffer, Rows, Scene, TreeInfo, check, load)
from . import _lib

SCREEN_WIDTH, SCREEN_HEIGHT, RAYS_PER_PIXEL, SEED = 640, 480, 4, 1984   # Constants.h:4-8, :458


def device_count() -> int:
    return load().bih_device_count()


def camera_reference(w: int, h: int) -> Camera:
    cam = Camera()
    check(load().bih_camera_reference(w, h, C.byref(cam)), "bih_camera_reference")
    return cam


def camera_ray_bound(cam: Camera) -> np.ndarray:
    """bih_camera_ray_bound: per-component bound of |D| over the camera's
    primary rays (host only; sizes the any-hit walk's miss-proof boxes)."""
    out = (C.c_float * 3)()
    check(load().bih_camera_ray_bound(C.byref(cam), out), "bih_camera_ray_bound")
    return np.array(out[:], np.float32)


class GPUArrayManager:
    """Scene + BIH on one device.  `tris` is a float32 (n, 9) soup."""

    def __init__(self, tris: np.ndarray, device: int = 0):
        self.tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
        self.scene = Scene(self.tris.shape[0], self.tris.ctypes.data)
        self.device = device
        self._tree = C.c_void_p()
        check(load().bih_build(C.byref(self.scene), device, C.byref(self._tree)), "bih_build")

    @classmethod
    def from_device(cls, ptr: int, n_tris: int, device: int = 0, stream: int | None = None):
        """Builds from a device-resident soup (e.g. a torch tensor's data_ptr())."""
        self = cls.__new__(cls)
        self.tris, self.scene, self.device = None, None, device
        self._tree = C.c_void_p()
        check(load().bih_build_device(C.c_void_p(ptr), n_tris, device, C.c_void_p(stream or 0),
                                      C.byref(self._tree)), "bih_build_device")
        return self

    @property
    def handle(self):
        return self._tree

    def rebuild(self):
        check(load().bih_rebuild(self._tree), "bih_rebuild")

    def info(self) -> TreeInfo:
        inf = TreeInfo()
        check(load().bih_tree_get_info(self._tree, C.byref(inf)), "bih_tree_get_info")
        return inf

    def set_param(self, param: int, value: int):
        """bih_tree_set_param (PARAM_*): work-order and test knobs; none changes a pixel."""
        check(load().bih_tree_set_param(self._tree, param, value), "bih_tree_set_param")

    def reserve(self, w: int, h: int, spp: int, rows: Rows | None = None, max_frames: int = 1):
        """bih_reserve: size every per-call buffer of renders of this shape (calls
        of up to max_frames frames) now, so that a frame loop allocates nothing."""
        check(load().bih_reserve(self._tree, w, h, spp, C.byref(rows) if rows is not None else None,
                                 max_frames), "bih_reserve")

    def bins_stats(self):
        """Frustum bins of the current camera and image (bih_bins_get_stats)."""
        from ._lib import BinsStats
        st = BinsStats()
        check(load().bih_bins_get_stats(self._tree, C.byref(st)), "bih_bins_get_stats")
        return st

    def export(self, which: int, dtype) -> np.ndarray:
        n = C.c_size_t(0)
        check(load().bih_tree_export(self._tree, which, None, C.byref(n)), "bih_tree_export")
        out = np.zeros(n.value // np.dtype(dtype).itemsize, dtype)
        check(load().bih_tree_export(self._tree, which, out.ctypes.data, C.byref(n)), "bih_tree_export")
        return out

    def arrays(self) -> dict:
        """Canonical arrays under the oracle's names (OracleTree attributes)."""
        a = {
            "morton": self.export(_lib.ARR_MORTON_SORTED, np.uint32),
            "tri_idx": self.export(_lib.ARR_TRI_INDEX, np.uint32),
            "unique_mc": self.export(_lib.ARR_UNIQUE_MC, np.uint32),
            "dup_cnt": self.export(_lib.ARR_DUP_COUNT, np.uint32),
            "first_idx": self.export(_lib.ARR_FIRST_IDX, np.int32),
            "leaf_parent": self.export(_lib.ARR_LEAF_PARENT, np.int32),
            "clip": self.export(_lib.ARR_CLIP, np.float32).reshape(-1, 2),
            "axis": self.export(_lib.ARR_AXIS, np.int32),
            "children": self.export(_lib.ARR_CHILDREN, np.int32).reshape(-1, 2),
            "is_leaf": self.export(_lib.ARR_IS_LEAF, np.uint8).reshape(-1, 2),
            "parent": self.export(_lib.ARR_PARENT, np.int32),
            "lo": self.export(_lib.ARR_TRI_LO, np.float32).reshape(-1, 3),
            "hi": self.export(_lib.ARR_TRI_HI, np.float32).reshape(-1, 3),
        }
        inf = self.info()
        a["scene_lo"] = np.array(inf.scene_lo[:], np.float32)
        a["scene_hi"] = np.array(inf.scene_hi[:], np.float32)
        return a

    def close(self):
        if getattr(self, "_tree", None) and self._tree.value:
            load().bih_free(self._tree)
            self._tree = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Renderer:
    """Per-frame renderer over a GPUArrayManager (Renderer::Render, Renderer.cpp:415)."""

    def __init__(self, arrays: GPUArrayManager, w: int = SCREEN_WIDTH, h: int = SCREEN_HEIGHT,
                 spp: int = RAYS_PER_PIXEL, seed: int = SEED, camera: Camera | None = None):
        self.arrays, self.w, self.h, self.spp, self.seed = arrays, w, h, spp, seed
        self.camera = camera if camera is not None else camera_reference(w, h)
        self.frame = 0

    def render(self, frame: int | None = None, rows: tuple[int, int] | None = None,
               out: np.ndarray | None = None) -> np.ndarray:
        """One frame into a host (h, w) uint32 image (0x00BBGGRR, row 0 = bottom).
        `out`: a caller-owned C-contiguous (nrows, w) uint32 framebuffer to render
        into (a frame loop reuses it; see host_register)."""
        f = self.frame if frame is None else frame
        row0, nrows = rows if rows is not None else (0, self.h)
        if out is None:
            out = np.zeros((nrows, self.w), np.uint32)
        elif out.shape != (nrows, self.w) or out.dtype != np.uint32 or not out.flags.c_contiguous:
            raise ValueError(f"out must be a C-contiguous ({nrows}, {self.w}) uint32 array")
        fb = Framebuffer(self.w, self.h, self.spp, f, self.seed, out.ctypes.data)
        sc = C.byref(self.arrays.scene) if self.arrays.scene is not None else None
        if rows is None:
            check(load().bih_render(sc, self.arrays.handle, C.byref(self.camera), C.byref(fb)), "bih_render")
        else:
            check(load().bih_render_rows(sc, self.arrays.handle, C.byref(self.camera), C.byref(fb),
                                         row0, nrows), "bih_render_rows")
        self.frame = f + 1
        return out

    def render_device(self, out_ptr: int, frame: int, rows: Rows | None = None,
                      traverse: int = TRAVERSE_ANYHIT, stats_ptr: int | None = None,
                      stream: int | None = None):
        """Asynchronous device-resident render into out_ptr (u32, nrows*w)."""
        check(load().bih_render_device(self.arrays.handle, C.byref(self.camera), self.w, self.h,
                                       self.spp, frame, self.seed,
                                       C.byref(rows) if rows is not None else None, traverse,
                                       C.c_void_p(out_ptr), C.c_void_p(stats_ptr or 0),
                                       C.c_void_p(stream or 0)), "bih_render_device")

    def render_device_frames(self, out_ptr: int, frame0: int, nframes: int, out_stride: int,
                             rows: Rows | None = None, stream: int | None = None):
        """Frames frame0 .. frame0+nframes-1 (any-hit) in one call
        (bih_render_device_frames); frame j at out_ptr + 4*j*out_stride bytes."""
        check(load().bih_render_device_frames(self.arrays.handle, C.byref(self.camera), self.w, self.h,
                                              self.spp, frame0, nframes, self.seed,
                                              C.byref(rows) if rows is not None else None,
                                              C.c_void_p(out_ptr), out_stride, C.c_void_p(stream or 0)),
              "bih_render_device_frames")

    def render_whitted(self, frame: int | None = None) -> np.ndarray:
        """Config C4: one frame of 8-bounce mirror rays (bih_render_whitted) into a
        host (h, w) uint32 image."""
        f = self.frame if frame is None else frame
        out = np.zeros((self.h, self.w), np.uint32)
        fb = Framebuffer(self.w, self.h, self.spp, f, self.seed, out.ctypes.data)
        sc = C.byref(self.arrays.scene) if self.arrays.scene is not None else None
        check(load().bih_render_whitted(sc, self.arrays.handle, C.byref(self.camera), C.byref(fb)),
              "bih_render_whitted")
        self.frame = f + 1
        return out

    def render_whitted_device(self, out_ptr: int, frame: int, rows: Rows | None = None,
                              hits_ptr: int | None = None, stream: int | None = None):
        """Asynchronous C4 render into out_ptr (u32, nrows*w); hits_ptr (optional,
        u32 per sample) receives each sample's hit count along its mirror path."""
        check(load().bih_render_whitted_device(self.arrays.handle, C.byref(self.camera), self.w, self.h,
                                               self.spp, frame, self.seed,
                                               C.byref(rows) if rows is not None else None,
                                               C.c_void_p(out_ptr), C.c_void_p(hits_ptr or 0),
                                               C.c_void_p(stream or 0)), "bih_render_whitted_device")

    def whitted_work(self) -> dict:
        """Per bounce d = 0..8 of the last Whitted render (run with
        PARAM_WHITTED_COUNTERS on): rays traced, BIH nodes entered, triangles
        tested (bih_whitted_work)."""
        n = 9
        rays, nodes, tris = (C.c_uint32 * n)(), (C.c_uint64 * n)(), (C.c_uint64 * n)()
        check(load().bih_whitted_work(self.arrays.handle, rays, nodes, tris), "bih_whitted_work")
        return {"rays": list(rays), "nodes": list(nodes), "tris": list(tris)}

    def render_history(self, n: int) -> np.ndarray:
        """(n, 3) ms {kernel start, kernel end, end of the render's work} of the
        last n renders (issued with set_timing on), after the oldest one's kernel
        start (bih_render_history)."""
        t = (C.c_double * (3 * n))()
        check(load().bih_render_history(self.arrays.handle, n, t), "bih_render_history")
        return np.array(t[:], np.float64).reshape(n, 3)

    def sync(self, stream: int | None = None):
        check(load().bih_sync(self.arrays.handle, C.c_void_p(stream or 0)), "bih_sync")

    def set_timing(self, on: bool = True):
        """Record device-time events around every render (bih_set_timing)."""
        check(load().bih_set_timing(self.arrays.handle, 1 if on else 0), "bih_set_timing")

    def last_render_ms(self) -> float:
        ms = C.c_double(0.0)
        check(load().bih_last_render_ms(self.arrays.handle, C.byref(ms)), "bih_last_render_ms")
        return ms.value

    def last_render_times(self) -> tuple[float, float]:
        """(main render kernel ms, ms of the render call's device work after it:
        k_render_fallback for frustum-bin renders)."""
        k, t = C.c_double(0.0), C.c_double(0.0)
        check(load().bih_last_render_times(self.arrays.handle, C.byref(k), C.byref(t)),
              "bih_last_render_times")
        return k.value, t.value


def host_register(arr: np.ndarray):
    """Page-locks a host framebuffer (bih_host_register) so that bih_render's
    device-to-host copy into it runs at DMA rate; host_unregister before it is
    freed."""
    check(load().bih_host_register(C.c_void_p(arr.ctypes.data), arr.nbytes), "bih_host_register")


def host_unregister(arr: np.ndarray):
    check(load().bih_host_unregister(C.c_void_p(arr.ctypes.data)), "bih_host_unregister")


def load_obj(path: str) -> np.ndarray:
    """Wavefront OBJ -> float32 (n, 9) soup in file order (bih_scene_load_obj;
    Model::LoadModel + App::LoadModels flattening, Model.cpp:10-95,
    App.cpp:65-121).  Raises BihError (BIH_ERR_IO / BIH_ERR_PARSE with the line)."""
    sc = Scene()
    line = C.c_uint32(0)
    rc = load().bih_scene_load_obj(os.fsencode(path), C.byref(sc), C.byref(line))
    if rc != _lib.BIH_OK:
        raise BihError(rc, f"bih_scene_load_obj({path!r})" + (f" line {line.value}" if line.value else ""))
    try:
        if sc.n_tris == 0:
            return np.zeros((0, 9), np.float32)
        return np.ctypeslib.as_array(C.cast(sc.v, C.POINTER(C.c_float)), (sc.n_tris, 9)).copy()
    finally:
        load().bih_scene_free(C.byref(sc))


class Model:
    """Model(path) (Model.h / Model.cpp:6-8): the triangles of one OBJ file."""

    def __init__(self, path: str):
        self.path = path
        self.triangles = load_obj(path)

    def __len__(self):
        return self.triangles.shape[0]


def unpack_rgba(img: np.ndarray) -> np.ndarray:
    """0x00BBGGRR -> (..., 4) uint8 RGBA (alpha byte as stored, 0)."""
    return img.astype("<u4").view(np.uint8).reshape(img.shape + (4,))


def write_ppm(path: str, img: np.ndarray):
    """PPM (P6) with row 0 at the bottom, as the GL quad shows it."""
    rgb = unpack_rgba(img)[::-1, :, :3]
    h, w = img.shape
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (w, h))
        f.write(np.ascontiguousarray(rgb).tobytes())


__all__ = ["GPUArrayManager", "Renderer", "Model", "load_obj", "host_register", "host_unregister", "Camera", "Rows", "BihError", "camera_reference",
           "camera_ray_bound", "device_count", "unpack_rgba", "write_ppm", "scenes", "TRAVERSE_ANYHIT",
           "TRAVERSE_REFERENCE", "PARAM_ITEM_TILES", "PARAM_PAIR_CAP", "PARAM_BINS_CAP", "PARAM_FORCE_FALLBACK",
           "PARAM_WHITTED_COUNTERS", "PARAM_STATIC_SOUP", "PARAM_TEST_ALLOC_FAIL"]
