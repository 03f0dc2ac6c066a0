#!/usr/bin/env python3
"""Kernel-only driver for rocprofv3: repeated BIH rebuilds of the bench soup."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--builds", type=int, default=10)
    a = ap.parse_args()
    import torch
    import bihrt
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    tris = bihrt.scenes.soup(a.tris, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=s.cuda_stream)
    ms = []
    for _ in range(a.builds):
        g.rebuild()
        ms.append(g.info().build_ms)
    print("build ms", [round(x, 3) for x in ms])


if __name__ == "__main__":
    main()
