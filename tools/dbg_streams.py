"""Diagnostic: frames on 2 streams (test_frames_in_flight_on_streams) with and
without a device sync after the output buffers are filled; per frame the
pixels that differ from the oracle and how many are still the fill value."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "bih-gpu-raytracer_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import torch
import bihrt
from oracle import oracle as O

sync_fill = int(sys.argv[1])
fill = int(sys.argv[2]) if len(sys.argv) > 2 else 0
tris = bihrt.scenes.soup(20_000, seed=9)
g = bihrt.GPUArrayManager(tris)
ot = O.OracleTree(tris)
w, h = 160, 96
r = bihrt.Renderer(g, w, h)
streams = [torch.cuda.Stream() for _ in range(2)]
frames = [0, 1, 2, 3, 7, 8, 9, 30, 31, 2, 3]
outs = [torch.full((h * w,), fill, dtype=torch.int32, device="cuda") for _ in frames]
if sync_fill:
    torch.cuda.synchronize()
for k, f in enumerate(frames):
    if k == 6:
        g.rebuild()
    r.render_device(outs[k].data_ptr(), f, stream=streams[k % 2].cuda_stream)
torch.cuda.synchronize()
for k, f in enumerate(frames):
    ref, _ = ot.render(w, h, frame=f)
    got = outs[k].cpu().numpy().view(np.uint32).reshape(h, w)
    bad = got != ref
    print("sync_fill", sync_fill, "k", k, "frame", f, "differ", int(bad.sum()),
          "fill-valued", int((got == np.uint32(fill & 0xFFFFFFFF)).sum()))
