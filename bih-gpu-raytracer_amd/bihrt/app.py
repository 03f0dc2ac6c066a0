"""Presentation-free frame loop.

Mirrors the reference application shell without windowing or GL interop:

  main()            src/Main.cpp:42-66   mesh name -> "resources/<name>/<name>.obj"
  App::LoadModels   src/App.cpp:65-164   -> App.load_models (bih_scene_load_obj +
                                            bih_build, host prep on the device)
  App::Run          src/App.cpp:170-187  -> App.run: per frame Renderer::Render
                                            = rebuild the BIH (Renderer.cpp:422-503)
                                            + cudaRender; prints FPS like
                                            Window::ShowFPS
  presentation      Renderer.cpp:644-670 -> PPM per frame (row 0 at the bottom,
                                            as the GL quad shows it)

usage:  python -m bihrt --mesh sponza --resources path/to/resources --frames 10 \
            --out frames/f%04d.ppm [--width 640 --height 480 --no-rebuild]
        python -m bihrt --obj file.obj ...     (explicit path)
        python -m bihrt --scene cornell|torus|soup[:N] ...   (built-in scenes)
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

from . import (RAYS_PER_PIXEL, SCREEN_HEIGHT, SCREEN_WIDTH, SEED, GPUArrayManager, Renderer,
               load_obj, scenes, write_ppm)


def mesh_path(resources: str, name: str) -> str:
    """Main.cpp:55: resources/<name>/<name>.obj"""
    return os.path.join(resources, name, name + ".obj")


def builtin_scene(spec: str) -> np.ndarray:
    name, _, n = spec.partition(":")
    if name == "cornell":
        return scenes.cornell()
    if name == "torus":
        return scenes.torus()
    if name == "soup":
        return scenes.soup(int(n) if n else 1_000_000, seed=1)
    raise ValueError(f"unknown scene {spec!r} (cornell | torus | soup[:N])")


class App:
    """App (src/App.h): owns the scene arrays and the renderer of one device."""

    def __init__(self, width: int = SCREEN_WIDTH, height: int = SCREEN_HEIGHT,
                 spp: int = RAYS_PER_PIXEL, seed: int = SEED, device: int = 0):
        self.width, self.height, self.spp, self.seed, self.device = width, height, spp, seed, device
        self.arrays = None
        self.renderer = None

    def load_models(self, tris_or_path) -> int:
        """App::LoadModels: flatten the model's triangles (file order), then
        build the BIH on the device.  Returns the triangle count."""
        tris = load_obj(tris_or_path) if isinstance(tris_or_path, str) else tris_or_path
        if tris.shape[0] == 0:
            raise ValueError("scene holds no triangles")
        self.arrays = GPUArrayManager(tris, device=self.device)
        self.renderer = Renderer(self.arrays, self.width, self.height, spp=self.spp, seed=self.seed)
        info = self.arrays.info()
        print(f"Loaded {tris.shape[0]} triangles...", flush=True)
        print("scene bbox lo: [%g, %g, %g]" % tuple(info.scene_lo), flush=True)
        print("scene bbox hi: [%g, %g, %g]" % tuple(info.scene_hi), flush=True)
        return tris.shape[0]

    def run(self, frames: int, out_pattern: str | None = None, rebuild: bool = True,
            every: int = 1):
        """App::Run for a fixed number of frames: Renderer::Render each frame
        (BIH rebuild + render), optional PPM output; returns the frames."""
        assert self.renderer is not None, "load_models first"
        imgs = []
        last = time.perf_counter()
        for f in range(frames):
            if rebuild and f > 0:
                self.arrays.rebuild()
            img = self.renderer.render(f)
            now = time.perf_counter()
            fps = 1.0 / max(now - last, 1e-9)
            last = now
            print(f"frame {f}: {fps:.1f} FPS (incl. host copy)", flush=True)
            if out_pattern and f % every == 0:
                path = out_pattern % f if "%" in out_pattern else out_pattern
                d = os.path.dirname(path)
                if d:
                    os.makedirs(d, exist_ok=True)
                write_ppm(path, img)
            imgs.append(img)
        return imgs


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m bihrt", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    src = ap.add_mutually_exclusive_group(required=True)
    src.add_argument("--mesh", help="mesh name: <resources>/<name>/<name>.obj (Main.cpp:55)")
    src.add_argument("--obj", help="explicit OBJ path")
    src.add_argument("--scene", help="built-in scene: cornell | torus | soup[:N]")
    ap.add_argument("--resources", default="resources")
    ap.add_argument("--width", type=int, default=SCREEN_WIDTH)
    ap.add_argument("--height", type=int, default=SCREEN_HEIGHT)
    ap.add_argument("--spp", type=int, default=RAYS_PER_PIXEL)
    ap.add_argument("--frames", type=int, default=1)
    ap.add_argument("--out", default=None, help="PPM path; '%%d' formats the frame number")
    ap.add_argument("--every", type=int, default=1, help="write every k-th frame")
    ap.add_argument("--no-rebuild", action="store_true",
                    help="build once (the reference rebuilds every frame)")
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)
    if a.mesh:
        path = mesh_path(a.resources, a.mesh)
        if not os.path.exists(path):
            print(f"File doesn't exist: {path}", file=sys.stderr)
            return 2
        scene = path
    elif a.obj:
        scene = a.obj
    else:
        scene = builtin_scene(a.scene)
    app = App(a.width, a.height, a.spp, device=a.device)
    app.load_models(scene)
    app.run(a.frames, a.out, rebuild=not a.no_rebuild, every=a.every)
    return 0
