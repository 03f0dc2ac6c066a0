#!/usr/bin/env python3
"""The bench's timed window (bench.py Workload.timed) replayed for a trace:
warm-up calls [warmup frames in calls of G, then one of each timed size],
then the timed calls [steps frames in calls of G] rotating over --streams
streams, optionally only rank q of Q's bands (--share q/Q).  Prints the host
clock (CLOCK_MONOTONIC ns, rocprofv3's clock) at the window's start, after
each call's issue and after the final synchronisation, so that
tools/window_timeline.py can place the kernels of a rocprofv3 kernel trace
of the same run on the host's window."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def call_sizes(n, g):
    out = [g] * (n // g)
    if n % g:
        out.append(n % g)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--group", type=int, default=16)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--share", default="", help="q/Q: rank q of Q's interleaved 8-row bands")
    ap.add_argument("--repeat", type=int, default=3, help="timed windows (each after its own warm-up)")
    a = ap.parse_args()
    import torch
    import bihrt
    from bihrt import tiling
    streams = [torch.cuda.Stream() for _ in range(a.streams)]
    torch.cuda.set_stream(streams[0])
    tris = bihrt.scenes.soup(1_000_000, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=streams[0].cuda_stream)
    W, H, G = 1920, 1080, a.group
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
    calls = call_sizes(a.steps, G)
    frame = 0
    for rep in range(a.repeat):
        warm = call_sizes(a.warmup, G)
        warm += [m for m in sorted(set(calls)) if m not in warm]
        while len(warm) < a.streams:
            warm.append(calls[0])
        c = 0

        def issue(m):
            nonlocal c, frame
            s = streams[c % a.streams]
            o = outs[c % a.streams].data_ptr()
            if m == 1:
                r.render_device(o, frame, rows=rows, stream=s.cuda_stream)
            else:
                r.render_device_frames(o, frame, m, stride, rows=rows, stream=s.cuda_stream)
            c += 1
            frame += m

        for m in warm:
            issue(m)
        torch.cuda.synchronize()
        t = [time.monotonic_ns()]
        for m in calls:
            issue(m)
            t.append(time.monotonic_ns())
        torch.cuda.synchronize()
        t.append(time.monotonic_ns())
        print("window", rep, "start_ns", t[0], "issued_ns", " ".join(str(x) for x in t[1:-1]), "end_ns", t[-1],
              "ms %.4f" % ((t[-1] - t[0]) / 1e6), "ms_per_frame %.5f" % ((t[-1] - t[0]) / 1e6 / a.steps), flush=True)


if __name__ == "__main__":
    main()
