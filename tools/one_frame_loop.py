#!/usr/bin/env python3
"""One frame per call on one stream (the bench's one_in_flight leg), for a
rocprofv3 kernel trace: per call the kernels and the gaps between them."""
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
    r = bihrt.Renderer(g, W, H, spp=4)
    g.reserve(W, H, 4, None, 1)
    out = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    for f in range(10):
        r.render_device(out.data_ptr(), f, stream=s.cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 40
    for f in range(10, 10 + n):
        r.render_device(out.data_ptr(), f, stream=s.cuda_stream)
    torch.cuda.synchronize()
    print("one-frame calls: %.4f ms each" % (1e3 * (time.perf_counter() - t0) / n))


if __name__ == "__main__":
    main()
