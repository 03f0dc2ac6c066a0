#!/usr/bin/env python3
"""Host time of each call of the with_rebuild loop (bih_rebuild, then the
render on the other streams in turn): where does the host wait?"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    import torch
    import bihrt
    from bihrt import tiling
    streams = [torch.cuda.Stream() for _ in range(3)]
    torch.cuda.set_stream(streams[0])
    tris = bihrt.scenes.soup(1_000_000, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=streams[0].cuda_stream)
    W, H = 1920, 1080
    g.set_param(bihrt.PARAM_STATIC_SOUP, int(os.environ.get("STATIC", "1")))
    r = bihrt.Renderer(g, W, H, spp=4)
    rows = tiling.band_rows(H, 8, 0, 1)
    g.reserve(W, H, 4, rows, 16)
    outs = [torch.zeros(H * W, dtype=torch.int32, device="cuda") for _ in streams]
    torch.cuda.synchronize()
    for rep in range(3):
        tr, tn = [], []
        for k in range(24):
            s = streams[1 + k % 2]
            t0 = time.perf_counter()
            if os.environ.get("CTX") == "1":
                with torch.cuda.stream(s):
                    g.rebuild()
                    t1 = time.perf_counter()
                    r.render_device(outs[1 + k % 2].data_ptr(), 3000 + 30 * rep + k, rows=rows,
                                    stream=s.cuda_stream)
            else:
                g.rebuild()
                t1 = time.perf_counter()
                r.render_device(outs[1 + k % 2].data_ptr(), 3000 + 30 * rep + k, rows=rows, stream=s.cuda_stream)
            t2 = time.perf_counter()
            tr.append(1e6 * (t1 - t0))
            tn.append(1e6 * (t2 - t1))
        torch.cuda.synchronize()
        print("rep", rep, "rebuild us", " ".join("%.0f" % x for x in tr[4:]))
        print("rep", rep, "render  us", " ".join("%.0f" % x for x in tn[4:]))


if __name__ == "__main__":
    main()
