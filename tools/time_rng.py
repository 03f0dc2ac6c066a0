#!/usr/bin/env python3
"""rocprofv3 driver for k_rng_init: re-seeds the per-pixel XORWOW states of
a 1080p frame --n times (frame 0 rendered again is a backward jump)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10)
    a = ap.parse_args()
    import torch
    import bihrt
    s = torch.cuda.Stream()
    g = bihrt.GPUArrayManager(bihrt.scenes.cornell())
    r = bihrt.Renderer(g, 1920, 1080)
    out = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
    for k in range(a.n):
        r.render_device(out.data_ptr(), 7 if k % 2 else 0, stream=s.cuda_stream)   # 0 -> 7 -> 0: re-seeds
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
