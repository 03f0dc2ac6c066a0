#!/usr/bin/env python3
"""Kernel-trace driver for one rank's share of the strong split: calls of
--group frames over band_rows(H, 8, rank, world) on --in-flight streams
(run under rocprofv3 --kernel-trace; prints wall ms per frame)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--group", type=int, default=16)
    ap.add_argument("--calls", type=int, default=40)
    ap.add_argument("--in-flight", type=int, default=3)
    a = ap.parse_args()
    import torch
    import bihrt
    from bihrt.tiling import band_rows
    W, H, G = 1920, 1080, a.group
    streams = [torch.cuda.Stream() for _ in range(a.in_flight)]
    tris = bihrt.scenes.soup(1_000_000, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=streams[0].cuda_stream)
    r = bihrt.Renderer(g, W, H)
    rows = band_rows(H, 8, a.rank, a.world) if a.world > 1 else None
    nrows = rows.nrows if rows is not None else H
    g.reserve(W, H, 4, rows if rows is not None else band_rows(H, 8, 0, 1), G)
    outs = [torch.zeros(G * nrows * W, dtype=torch.int32, device="cuda") for _ in streams]
    for k in range(6):
        j = k % len(streams)
        r.render_device_frames(outs[j].data_ptr(), k * G, G, nrows * W, rows=rows, stream=streams[j].cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.calls):
        j = k % len(streams)
        r.render_device_frames(outs[j].data_ptr(), (6 + k) * G, G, nrows * W, rows=rows,
                               stream=streams[j].cuda_stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print("ms_per_frame", 1e3 * el / (a.calls * G))


if __name__ == "__main__":
    main()
