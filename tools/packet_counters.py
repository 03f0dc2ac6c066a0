#!/usr/bin/env python3
"""Packet-level walk counters of a BIH_PACKET_COUNTERS=1 library build
(BIH_LIB=...): renders one bench frame per traversal; the library prints the
counters to stderr from bih_sync."""
import os
import sys

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
    r = bihrt.Renderer(g, 1920, 1080, spp=4)
    out = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
    for name, trav in (("anyhit", bihrt.TRAVERSE_ANYHIT), ("reference", bihrt.TRAVERSE_REFERENCE)):
        print(name, flush=True)
        sys.stdout.flush()
        r.render_device(out.data_ptr(), 0, traverse=trav, stream=s.cuda_stream)
        r.sync(s.cuda_stream)


if __name__ == "__main__":
    main()
