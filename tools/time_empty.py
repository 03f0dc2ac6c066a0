#!/usr/bin/env python3
"""Frame time of the bench workload with the reference camera and with the
camera turned away from the scene (every packet dead): the fixed per-packet
cost of ray setup, tile queue and writeback."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    import torch
    import bihrt
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    tris = bihrt.scenes.soup(1_000_000, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=s.cuda_stream)
    W, H = 1920, 1080
    cam = bihrt.camera_reference(W, H)
    away = bihrt.camera_reference(W, H)
    away.lower_left[2] = away.origin[2] - 1.0     # D.z = -1: every ray leaves the scene behind
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    for name, c in (("reference", cam), ("away", away)):
        r = bihrt.Renderer(g, W, H, spp=4, camera=c)
        for f in range(5):
            r.render_device(out.data_ptr(), f, stream=s.cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 50
        for f in range(5, 5 + n):
            r.render_device(out.data_ptr(), f, stream=s.cuda_stream)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / n * 1e3
        hit = int((out.cpu().numpy() != 0x281414).sum())
        print(f"{name}: {ms:.3f} ms per frame (one stream), non-background pixels {hit}", flush=True)


if __name__ == "__main__":
    main()
