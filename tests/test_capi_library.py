"""The C-ABI shared object loads, exports every include/bih.h entry point and
behaves on a host without a GPU (no compute calls here)."""
import ctypes as C
import subprocess

import numpy as np
import pytest


def test_exports_every_declared_symbol(bihrt_mod):
    from bihrt import _lib
    names = _lib.exported_symbols_from_header()
    assert len(names) >= 15, names
    L = _lib.load()
    for n in names:
        assert hasattr(L, n), f"{n} declared in include/bih.h but not exported"
    # and dynamically exported as C symbols (no C++ mangling)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for n in names:
        assert n in syms, n


def test_library_is_gfx950(bihrt_mod):
    from bihrt import _lib
    out = subprocess.run(["strings", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "gfx950" in out


def test_camera_reference_matches_oracle(bihrt_mod, oracle_mod):
    for w, h in [(640, 480), (1920, 1080), (256, 256), (3840, 2160), (37, 29)]:
        cam = bihrt_mod.camera_reference(w, h).as_list()
        ref = oracle_mod.camera_reference(w, h)
        assert np.array_equal(np.array(cam, np.float32).view(np.uint32), ref.view(np.uint32))
    c = bihrt_mod.camera_reference(640, 480).as_list()
    assert c[:3] == [2.0, 0.0, -2.0] and c[3:6] == [0.0, -1.0, -1.0]
    assert np.float32(c[6]) == np.float32(np.float32(640) / np.float32(480)) * 2


def test_errors_without_device(bihrt_mod):
    L = bihrt_mod._lib.load()
    assert L.bih_abi_version() == 4
    assert L.bih_strerror(-2).decode().startswith("no HIP device")
    assert L.bih_strerror(12345).decode() == "unknown error"
    cam = bihrt_mod.Camera()
    assert L.bih_camera_reference(0, 10, C.byref(cam)) == -1
    if bihrt_mod.device_count() == 0:
        tris = bihrt_mod.scenes.cornell()
        with pytest.raises(bihrt_mod.BihError) as e:
            bihrt_mod.GPUArrayManager(tris)
        assert e.value.code == -2
    # invalid arguments are rejected before touching a device
    t = C.c_void_p()
    assert L.bih_build(None, 0, C.byref(t)) == -1
    sc = bihrt_mod._lib.Scene(1 << 28, 1)
    assert L.bih_build(C.byref(sc), 0, C.byref(t)) == -6
    assert L.bih_render(None, None, None, None) == -1
    assert L.bih_render_device(None, None, 1, 1, 1, 0, 0, None, 0, None, None, None) == -1
    assert L.bih_reserve(None, 1920, 1080, 4, None, 16) == -1
    assert L.bih_tree_set_param(None, bihrt_mod.PARAM_ITEM_TILES, 1) == -1
    assert L.bih_tree_set_param(None, bihrt_mod.PARAM_STATIC_SOUP, 1) == -1
    # ABI 4: host framebuffer registration and the render history
    assert L.bih_host_register(None, 16) == -1
    assert L.bih_host_unregister(None) == -1
    hist = (C.c_double * 9)()
    assert L.bih_render_history(None, 3, hist) == -1
    if bihrt_mod.device_count() == 0:
        buf = np.zeros(1024, np.uint32)
        assert L.bih_host_register(C.c_void_p(buf.ctypes.data), buf.nbytes) == -2
    # the tree-info struct carries the allocation counter (ABI 2)
    assert bihrt_mod._lib.TreeInfo.device_allocs.offset + 8 == C.sizeof(bihrt_mod._lib.TreeInfo)


def test_no_cpu_fallback_in_product():
    """The product package never imports the oracle."""
    import os
    import re
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "bih-gpu-raytracer_amd")
    for dp, _, fs in os.walk(root):
        for f in fs:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                src = open(os.path.join(dp, f), errors="ignore").read()
                assert not re.search(r"^\s*(import|from)\s+oracle", src, re.M), f
                assert "bih_oracle" not in src, f
