"""Frame loop (bihrt.app): Main.cpp's mesh-path convention,
App::LoadModels -> App::Run with a per-frame BIH rebuild, PPM output.  The
GPU test renders an OBJ through the C ABI and checks every frame against the
oracle render of the same soup."""
import os

import numpy as np
import pytest


def test_mesh_path_convention(bihrt_mod):
    from bihrt.app import mesh_path
    assert mesh_path("resources", "sponza") == os.path.join("resources", "sponza", "sponza.obj")


def test_missing_mesh_exits_2(bihrt_mod, tmp_path, capsys):
    from bihrt.app import main
    assert main(["--mesh", "bunny", "--resources", str(tmp_path)]) == 2
    assert "doesn't exist" in capsys.readouterr().err


def test_ppm_writer_flips_rows(bihrt_mod, tmp_path):
    img = np.array([[0x000000FF, 0x0000FF00], [0x00FF0000, 0x00102030]], np.uint32)
    p = str(tmp_path / "a.ppm")
    bihrt_mod.write_ppm(p, img)
    data = open(p, "rb").read()
    assert data.startswith(b"P6\n2 2\n255\n")
    px = np.frombuffer(data[len(b"P6\n2 2\n255\n"):], np.uint8).reshape(2, 2, 3)
    # row 0 of the framebuffer is the bottom row of the picture
    assert px[1, 0].tolist() == [255, 0, 0] and px[0, 1].tolist() == [0x30, 0x20, 0x10]


@pytest.mark.gpu
def test_app_renders_obj_frames_like_the_oracle(gpu, bihrt_mod, oracle_mod, tmp_path):
    from bihrt import scenes as S
    from bihrt.app import App, main
    res = tmp_path / "resources"
    (res / "box").mkdir(parents=True)
    S.write_obj(str(res / "box" / "box.obj"), S.cornell(), shared=True)
    tris = bihrt_mod.load_obj(str(res / "box" / "box.obj"))
    app = App(96, 64)
    assert app.load_models(str(res / "box" / "box.obj")) == tris.shape[0]
    frames = app.run(3, str(tmp_path / "out" / "f%02d.ppm"))
    ot = oracle_mod.OracleTree(tris)
    for f, img in enumerate(frames):
        ref, _ = ot.render(96, 64, frame=f)
        assert np.array_equal(img, ref), f
        assert os.path.exists(tmp_path / "out" / f"f{f:02d}.ppm")
    assert main(["--mesh", "box", "--resources", str(res), "--width", "32", "--height", "16",
                 "--frames", "2"]) == 0
