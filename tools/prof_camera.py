#!/usr/bin/env python3
"""rocprofv3 driver for the per-camera cost: renders --frames frames of the
bench workload with the camera moving every frame (8 cameras in turn, as
bench.py's moving_camera leg), one stream."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--tris", type=int, default=1_000_000)
    a = ap.parse_args()
    import torch
    import bihrt
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    tris = bihrt.scenes.soup(a.tris, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=s.cuda_stream)
    r = bihrt.Renderer(g, 1920, 1080)
    base = r.camera.as_list()
    cams = []
    for k in range(8):
        c = list(base)
        for j, dj in enumerate((0.002 * k, 0.001 * k, -0.003 * k)):
            c[j] += dj
            c[3 + j] += dj
        cams.append(bihrt.Camera.from_list(c))
    out = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
    for f in range(a.frames):
        r.camera = cams[f % 8]
        r.render_device(out.data_ptr(), f, stream=s.cuda_stream)
    torch.cuda.synchronize()
    print("frames", a.frames, "done")


if __name__ == "__main__":
    main()
