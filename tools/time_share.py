#!/usr/bin/env python3
"""Per-frame cost of one rank's share of a row-band split (--world ranks):
wall ms per frame with frames in flight, host microseconds per render call
(issue cost, no sync), and the same for the full frame."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--in-flight", type=int, default=3)
    ap.add_argument("--rank", type=int, default=0)
    a = ap.parse_args()
    import torch
    import bihrt
    from bihrt.tiling import band_rows
    W, H = 1920, 1080
    streams = [torch.cuda.Stream() for _ in range(a.in_flight)]
    tris = bihrt.scenes.soup(1_000_000, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=streams[0].cuda_stream)
    r = bihrt.Renderer(g, W, H)
    outs = [torch.zeros(W * H, dtype=torch.int32, device="cuda") for _ in streams]
    res = {}
    for name, rows in (("full", None), ("share", band_rows(H, 8, a.rank, a.world))):
        base = 1000 if name == "full" else 5000
        for k in range(20):
            r.render_device(outs[k % len(streams)].data_ptr(), base + k, rows=rows,
                            stream=streams[k % len(streams)].cuda_stream)
        torch.cuda.synchronize()
        host = 0.0
        t0 = time.perf_counter()
        for k in range(a.frames):
            j = k % len(streams)
            h0 = time.perf_counter()
            r.render_device(outs[j].data_ptr(), base + 20 + k, rows=rows, stream=streams[j].cuda_stream)
            host += time.perf_counter() - h0
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        r.set_timing(True)
        r.render_device(outs[0].data_ptr(), base + 20 + a.frames, rows=rows, stream=streams[0].cuda_stream)
        torch.cuda.synchronize()
        kms, tail = r.last_render_times()
        r.set_timing(False)
        res[name] = {"ms_per_frame": 1e3 * el / a.frames, "host_us_per_call": 1e6 * host / a.frames,
                     "last_kernel_ms": kms, "last_tail_ms": tail}
    res["projected_efficiency"] = res["full"]["ms_per_frame"] / (a.world * res["share"]["ms_per_frame"])
    print(json.dumps(res))


if __name__ == "__main__":
    main()
