#!/usr/bin/env python3
"""Wave timeline of the packet kernel (BIH_WAVE_TIMELINE=1 library via
BIH_LIB): renders --frames frames of the bench workload one at a time and
lets bih_sync print each frame's per-wave summary to stderr."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--tris", type=int, default=1_000_000)
    a = ap.parse_args()
    import torch
    import bihrt
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    tris = bihrt.scenes.soup(a.tris, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=s.cuda_stream)
    r = bihrt.Renderer(g, 1920, 1080, spp=4)
    out = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
    for f in range(a.frames):
        r.render_device(out.data_ptr(), f, stream=s.cuda_stream)
        r.sync(s.cuda_stream)


if __name__ == "__main__":
    main()
