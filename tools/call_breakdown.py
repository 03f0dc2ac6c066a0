#!/usr/bin/env python3
"""Per-call cost breakdown of the render path (run under rocprofv3 --kernel-trace).

Renders `--calls` calls of `--frames` frames of the bench workload (1M soup,
1920x1080x4 by default), optionally only rank q of Q's interleaved 8-row bands
(`--share q/Q`), each call followed by a host synchronisation (`--sync 1`, the
isolated-launch shape) or all calls in flight on `--streams` streams.  Prints
the host wall time per call.  The kernel trace of the same run is split into
calls by tools/call_timeline.py: advance, gaps, render, fallback per call.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=40)
    ap.add_argument("--warm", type=int, default=8)
    ap.add_argument("--frames", type=int, default=1)
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--share", default="", help="q/Q: render rank q of Q's interleaved 8-row bands")
    ap.add_argument("--sync", type=int, default=1, help="synchronise after every call")
    ap.add_argument("--streams", type=int, default=1)
    a = ap.parse_args()
    import torch
    import bihrt
    from bihrt import tiling
    streams = [torch.cuda.Stream() for _ in range(a.streams)]
    torch.cuda.set_stream(streams[0])
    tris = bihrt.scenes.soup(a.tris, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=streams[0].cuda_stream)
    W, H, G = a.width, a.height, a.frames
    r = bihrt.Renderer(g, W, H, spp=4)
    if a.share:
        q, Q = (int(x) for x in a.share.split("/"))
        rows = tiling.band_rows(H, 8, q, Q)
    else:
        rows = tiling.band_rows(H, 8, 0, 1)
    g.reserve(W, H, 4, rows, G)
    stride = rows.nrows * W
    outs = [torch.zeros(G * stride, dtype=torch.int32, device="cuda") for _ in streams]
    torch.cuda.synchronize()

    def call(k):
        s = streams[k % len(streams)]
        o = outs[k % len(streams)].data_ptr()
        if G == 1:
            r.render_device(o, k, rows=rows, stream=s.cuda_stream)
        else:
            r.render_device_frames(o, k * G, G, stride, rows=rows, stream=s.cuda_stream)

    for k in range(a.warm):
        call(k)
        r.sync(streams[k % len(streams)].cuda_stream)
    times = []
    t00 = time.perf_counter()
    for k in range(a.warm, a.warm + a.calls):
        t0 = time.perf_counter()
        call(k)
        if a.sync:
            r.sync(streams[k % len(streams)].cuda_stream)   # bih_sync (diagnostic builds dump here)
        times.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    tot = time.perf_counter() - t00
    times.sort()
    print(f"calls {a.calls} x {G} frames share '{a.share}' sync {a.sync} streams {a.streams}: "
          f"wall per call median {1e3 * times[len(times) // 2]:.4f} ms, min {1e3 * times[0]:.4f} ms, "
          f"total {1e3 * tot / a.calls:.4f} ms per call, {1e3 * tot / (a.calls * G):.4f} ms per frame",
          flush=True)


if __name__ == "__main__":
    main()
