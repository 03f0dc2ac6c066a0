#!/usr/bin/env python3
"""Host cost of the with_rebuild step (bench.py's leg: bih_rebuild + a
one-frame render on rotating streams): per-call host microseconds of
rebuild and render without synchronising, and the wall time per step."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--in-flight", type=int, default=3)
    ap.add_argument("--static", type=int, default=1, help="BIH_PARAM_STATIC_SOUP (asynchronous rebuilds)")
    ap.add_argument("--render", type=int, default=1, help="0: rebuilds only")
    a = ap.parse_args()
    import torch
    import bihrt
    W, H = 1920, 1080
    streams = [torch.cuda.Stream() for _ in range(a.in_flight)]
    tris = bihrt.scenes.soup(1_000_000, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=streams[0].cuda_stream)
    g.set_param(bihrt.PARAM_STATIC_SOUP, a.static)
    r = bihrt.Renderer(g, W, H)
    outs = [torch.zeros(W * H, dtype=torch.int32, device="cuda") for _ in streams]

    def run(n, k0, record):
        tb = tr = 0.0
        for k in range(k0, k0 + n):
            j = k % len(streams)
            t0 = time.perf_counter()
            g.rebuild()
            t1 = time.perf_counter()
            if a.render:
                r.render_device(outs[j].data_ptr(), k, stream=streams[j].cuda_stream)
            t2 = time.perf_counter()
            tb += t1 - t0
            tr += t2 - t1
        return tb, tr

    run(20, 0, False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tb, tr = run(a.steps, 20, True)
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    n = a.steps
    print("host us per step: rebuild %.1f render %.1f total %.1f | wall us per step %.1f"
          % (1e6 * tb / n, 1e6 * tr / n, 1e6 * th / n, 1e6 * el / n))


if __name__ == "__main__":
    main()
