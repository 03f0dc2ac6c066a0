"""A compiled C caller of include/bih.h (tests/c/abi_smoke.c): gcc, C11,
-Werror, linked against libbih_amd.so -- the way the reference's host code
would bind the boundary in place of Renderer::Render (src/Renderer.cpp:415)
and Launch_cudaRender (src/CUDAKernels.cu:425-447)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

SRC = os.path.join(ROOT, "tests", "c", "abi_smoke.c")
LIBDIR = os.path.join(ROOT, "bih-gpu-raytracer_amd", "lib")


def _build(tmp_path) -> str:
    exe = str(tmp_path / "abi_smoke")
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-pedantic",
                    "-I", os.path.join(ROOT, "include"), SRC, "-o", exe,
                    "-L", LIBDIR, "-lbih_amd", "-Wl,-rpath," + LIBDIR,
                    "-Wl,-rpath-link,/opt/rocm/lib"], check=True)
    return exe


def test_c_caller_compiles_and_error_paths(tmp_path, bihrt_mod):
    """Header compiles as strict C11 and links; every device-free error path
    returns its documented code (no exit, no abort)."""
    bihrt_mod._lib.load()   # ensures the library is built
    exe = _build(tmp_path)
    r = subprocess.run([exe, "--errors"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "FAIL" not in r.stdout and r.stdout.count("ok ") >= 8, r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("fname,scene,w,h,frame", [
    ("cornell_256x256_f7.npy", "cornell", 256, 256, 7),
    ("bih1_dodeca_640x480_f0.npy", "bih1_dodeca", 640, 480, 0)])
def test_c_caller_renders_golden(fname, scene, w, h, frame, tmp_path, gpu, bihrt_mod):
    """bih_build -> bih_camera_reference -> bih_render (frames 0..F on the
    persistent RNG state) from C equals the committed golden framebuffer;
    bih_render_rows and bih_rebuild likewise; error codes with a live tree."""
    from conftest import edge_scenes
    exe = _build(tmp_path)
    tris = np.ascontiguousarray(edge_scenes()[scene], np.float32)
    sp, gp = tmp_path / "scene.f32", tmp_path / "golden.u32"
    tris.tofile(sp)
    np.ascontiguousarray(np.load(os.path.join(GOLDEN, fname)), np.uint32).tofile(gp)
    r = subprocess.run([exe, str(sp), str(tris.shape[0]), str(w), str(h), str(frame), str(gp)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "abi_smoke OK" in r.stdout, r.stdout + r.stderr
