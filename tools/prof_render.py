#!/usr/bin/env python3
"""Kernel-only driver for rocprofv3: builds the bench scene once and renders
`--frames` frames of the bench workload (default 1M soup, 1920x1080x4)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--traverse", choices=["anyhit", "reference"], default="anyhit")
    ap.add_argument("--group", type=int, default=1,
                    help="frames per render call (bih_render_device_frames; any-hit only)")
    ap.add_argument("--streams", type=int, default=1,
                    help="calls rotate over this many streams (the bench's headline shape: 3)")
    a = ap.parse_args()
    import torch
    import bihrt
    streams = [torch.cuda.Stream() for _ in range(a.streams)]
    s = streams[0]
    torch.cuda.set_stream(s)
    tris = bihrt.scenes.soup(a.tris, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0], stream=s.cuda_stream)
    r = bihrt.Renderer(g, a.width, a.height, spp=a.spp)
    P = a.width * a.height
    out = torch.zeros(a.group * P, dtype=torch.int32, device="cuda")
    trav = bihrt.TRAVERSE_ANYHIT if a.traverse == "anyhit" else bihrt.TRAVERSE_REFERENCE
    outs = [out] + [torch.zeros(a.group * P, dtype=torch.int32, device="cuda") for _ in streams[1:]]
    for f in range(a.frames):     # --frames render calls
        s, o = streams[f % len(streams)], outs[f % len(streams)]
        if a.group > 1 and trav == bihrt.TRAVERSE_ANYHIT:
            r.render_device_frames(o.data_ptr(), f * a.group, a.group, P, stream=s.cuda_stream)
        else:
            r.render_device(o.data_ptr(), f, traverse=trav, stream=s.cuda_stream)
    torch.cuda.synchronize()
    print("frames", a.frames, "done")


if __name__ == "__main__":
    main()
