#!/usr/bin/env python3
"""The bench's with_rebuild leg replayed for a trace: per step bih_rebuild
(the tree's stream, streams[0]) then a one-frame render on streams 1 and 2 in
turn; `--steps` timed steps after 8 warm-up steps; prints the host window
like tools/window_trace.py (for tools/window_timeline.py)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--repeat", type=int, default=2)
    a = ap.parse_args()
    import torch
    import bihrt
    from bihrt import tiling
    streams = [torch.cuda.Stream() for _ in range(3)]
    torch.cuda.set_stream(streams[0])
    tris = bihrt.scenes.soup(1_000_000, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=streams[0].cuda_stream)
    W, H = 1920, 1080
    g.set_param(bihrt.PARAM_STATIC_SOUP, 1)   # as the bench: rebuilds without a host synchronisation
    r = bihrt.Renderer(g, W, H, spp=4)
    rows = tiling.band_rows(H, 8, 0, 1)
    g.reserve(W, H, 4, rows, 16)
    outs = [torch.zeros(H * W, dtype=torch.int32, device="cuda") for _ in streams]
    torch.cuda.synchronize()
    k = 0

    def step():
        nonlocal k
        s = streams[1 + k % 2]
        with torch.cuda.stream(s):
            g.rebuild()
            r.render_device(outs[1 + k % 2].data_ptr(), 2000 + k, rows=rows, stream=s.cuda_stream)
        k += 1

    for rep in range(a.repeat):
        for _ in range(8):
            step()
        torch.cuda.synchronize()
        t = [time.monotonic_ns()]
        for _ in range(a.steps):
            step()
            t.append(time.monotonic_ns())
        torch.cuda.synchronize()
        t.append(time.monotonic_ns())
        print("window", rep, "start_ns", t[0], "issued_ns", " ".join(str(x) for x in t[1:-1]), "end_ns", t[-1],
              "ms %.4f" % ((t[-1] - t[0]) / 1e6), "ms_per_step %.5f" % ((t[-1] - t[0]) / 1e6 / a.steps), flush=True)


if __name__ == "__main__":
    main()
