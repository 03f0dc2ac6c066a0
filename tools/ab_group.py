#!/usr/bin/env python3
"""A/B timing of the bench headline loop (library via BIH_LIB): calls of
--group consecutive frames on --in-flight streams, ms per frame, plus the
device time of one isolated call (bih_last_render_times)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=800)
    ap.add_argument("--group", type=int, default=8)
    ap.add_argument("--in-flight", type=int, default=3)
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bihrt
    W, H, G = a.width, a.height, a.group
    streams = [torch.cuda.Stream() for _ in range(a.in_flight)]
    tris = bihrt.scenes.soup(a.tris, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=streams[0].cuda_stream)
    r = bihrt.Renderer(g, W, H)
    outs = [torch.zeros(G * W * H, dtype=torch.int32, device="cuda") for _ in streams]
    calls = a.frames // G
    for k in range(6):
        r.render_device_frames(outs[k % len(streams)].data_ptr(), k * G, G, W * H,
                               stream=streams[k % len(streams)].cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(calls):
        r.render_device_frames(outs[k % len(streams)].data_ptr(), (6 + k) * G, G, W * H,
                               stream=streams[k % len(streams)].cuda_stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    r.set_timing(True)
    kms = []
    for k in range(5):
        r.render_device_frames(outs[0].data_ptr(), (6 + calls + k) * G, G, W * H, stream=streams[0].cuda_stream)
        torch.cuda.synchronize()
        kms.append(r.last_render_times()[0])
    img = outs[0][: W * H].cpu().numpy().view(np.uint32)
    print(json.dumps({"lib": os.path.basename(os.environ.get("BIH_LIB", "") or "default"),
                      "ms_per_frame": 1e3 * el / (calls * G), "kernel_ms_per_frame": sum(kms) / len(kms) / G,
                      "img_hash": int(img.astype(np.uint64).sum())}), flush=True)


if __name__ == "__main__":
    main()
