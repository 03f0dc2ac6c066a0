#!/usr/bin/env python3
"""Prints the shortcut/bin counters of a BIH_FAST_COUNTERS=1 library variant
(BIH_LIB=...): renders --frames frames of the bench workload, bih_sync after
each (the library prints the counters of the last render to stderr)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--group", type=int, default=1, help="frames per call (bih_render_device_frames)")
    ap.add_argument("--scene", default="soup", choices=["soup", "torus"])
    a = ap.parse_args()
    import torch
    import bihrt
    s = torch.cuda.Stream()
    tris = bihrt.scenes.soup(a.tris, seed=1) if a.scene == "soup" else bihrt.scenes.torus()
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=s.cuda_stream)
    r = bihrt.Renderer(g, a.width, a.height)
    P = a.width * a.height
    out = torch.zeros(P * a.group, dtype=torch.int32, device="cuda")
    for f in range(a.frames):
        if a.group > 1:
            r.render_device_frames(out.data_ptr(), f * a.group, a.group, P, stream=s.cuda_stream)
        else:
            r.render_device(out.data_ptr(), f, stream=s.cuda_stream)
        r.sync(s.cuda_stream)
    st = g.bins_stats()
    print("scene %s bins: %s" % (a.scene, {k: getattr(st, k) for k, _ in st._fields_}), flush=True)


if __name__ == "__main__":
    main()
