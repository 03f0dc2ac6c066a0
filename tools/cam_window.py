#!/usr/bin/env python3
"""The bench's moving_camera leg replayed for a trace: 8 cameras in turn, one
frame per step on --streams rotating streams, `--steps` timed steps after 8
warm-up steps; prints the host window like tools/window_trace.py (for
tools/window_timeline.py)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--repeat", type=int, default=2)
    a = ap.parse_args()
    import torch
    import bihrt
    from bihrt import Camera, tiling
    streams = [torch.cuda.Stream() for _ in range(a.streams)]
    torch.cuda.set_stream(streams[0])
    tris = bihrt.scenes.soup(1_000_000, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=streams[0].cuda_stream)
    W, H = 1920, 1080
    r = bihrt.Renderer(g, W, H, spp=4)
    rows = tiling.band_rows(H, 8, 0, 1)
    g.reserve(W, H, 4, rows, 16)
    base = r.camera.as_list()
    cams = []
    for k in range(8):
        c = list(base)
        dd = (0.002 * k, 0.001 * k, -0.003 * k)
        for j in range(3):
            c[j] += dd[j]
            c[3 + j] += dd[j]
        cams.append(Camera.from_list(c))
    outs = [torch.zeros(H * W, dtype=torch.int32, device="cuda") for _ in streams]
    torch.cuda.synchronize()
    k = 0

    def step():
        nonlocal k
        r.camera = cams[k % len(cams)]
        s = streams[k % a.streams]
        r.render_device(outs[k % a.streams].data_ptr(), 6000 + k, rows=rows, stream=s.cuda_stream)
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
