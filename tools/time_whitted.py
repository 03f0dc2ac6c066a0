#!/usr/bin/env python3
"""Times config C4 (8-bounce Whitted, bih_render_whitted_device) on the bench
soup: ms per frame, primary and total rays per second."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--frames", type=int, default=10)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bihrt
    s = torch.cuda.Stream()
    tris = bihrt.scenes.soup(a.tris, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=s.cuda_stream)
    r = bihrt.Renderer(g, a.width, a.height)
    r.set_timing(True)
    P = a.width * a.height
    out = torch.zeros(P, dtype=torch.int32, device="cuda")
    hits = torch.zeros(P * 4, dtype=torch.int32, device="cuda")
    r.render_whitted_device(out.data_ptr(), 0, hits_ptr=hits.data_ptr(), stream=s.cuda_stream)
    torch.cuda.synchronize()
    h = hits.to(torch.int64)
    traced = int(torch.clamp(h + 1, max=9).sum())
    hist = torch.bincount(hits.view(-1), minlength=10).tolist()
    t0 = time.perf_counter()
    for f in range(1, a.frames + 1):
        r.render_whitted_device(out.data_ptr(), f, stream=s.cuda_stream)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / a.frames
    k, tail = r.last_render_times()
    print(json.dumps({"ms_per_frame": el * 1e3, "trace_ms_last": k, "primary_rays_per_s": P * 4 / el,
                      "rays_traced_frame0": traced, "rays_traced_per_s": traced / el,
                      "hit_histogram": hist}))


if __name__ == "__main__":
    main()
