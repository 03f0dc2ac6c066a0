#!/usr/bin/env python3
"""The builder alone: `--n` rebuilds of the 1M soup back to back on the
tree's stream (BIH_PARAM_STATIC_SOUP: no host wait), for a rocprofv3 kernel
trace of the build chain without renders beside it."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=30)
    ap.add_argument("--tris", type=int, default=1_000_000)
    a = ap.parse_args()
    import torch
    import bihrt
    tris = bihrt.scenes.soup(a.tris, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0])
    g.set_param(bihrt.PARAM_STATIC_SOUP, 1)
    g.rebuild()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.n):
        g.rebuild()
    torch.cuda.synchronize()
    print("rebuilds", a.n, "ms each %.4f" % (1e3 * (time.perf_counter() - t0) / a.n), "build_ms", g.info().build_ms)


if __name__ == "__main__":
    main()
