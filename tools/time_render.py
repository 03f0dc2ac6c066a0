#!/usr/bin/env python3
"""Times the render kernel (HIP events on the render stream) for A/B runs.
Library variant via BIH_LIB, kernel variant via BIH_RENDER_KERNEL."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--traverse", choices=["anyhit", "reference"], default="anyhit")
    ap.add_argument("--tag", default="")
    ap.add_argument("--world", type=int, default=1, help="render rank 0's interleaved bands of W ranks")
    ap.add_argument("--band", type=int, default=8)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bihrt
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    tris = bihrt.scenes.soup(a.tris, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=s.cuda_stream)
    r = bihrt.Renderer(g, a.width, a.height, spp=a.spp)
    out = torch.zeros(a.width * a.height, dtype=torch.int32, device="cuda")
    from bihrt.tiling import band_rows
    rows = band_rows(a.height, a.band, 0, a.world) if a.world > 1 else None
    trav = bihrt.TRAVERSE_ANYHIT if a.traverse == "anyhit" else bihrt.TRAVERSE_REFERENCE
    ms = []
    for f in range(a.warmup + a.frames):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        r.render_device(out.data_ptr(), f, rows=rows, traverse=trav, stream=s.cuda_stream)
        e1.record(s)
        if f >= a.warmup:
            ms.append((e0, e1))
    torch.cuda.synchronize()
    t = [x.elapsed_time(y) for x, y in ms]
    img = out.cpu().numpy().view(np.uint32)
    print(json.dumps({"tag": a.tag, "lib": os.environ.get("BIH_LIB", "default"),
                      "kernel": os.environ.get("BIH_RENDER_KERNEL", "default"),
                      "traverse": a.traverse, "world": a.world, "ms_mean": sum(t) / len(t), "ms_min": min(t),
                      "ms_median": sorted(t)[len(t) // 2], "ms_all": [round(x, 3) for x in t],
                      "mrays_s": a.width * a.height * a.spp / (sum(t) / len(t)) / 1e3,
                      "img_hash": int(img.astype(np.uint64).sum())}), flush=True)


if __name__ == "__main__":
    main()
