"""Times the steps of tests/test_whitted.py::test_whitted_4k_properties on the
GPU (diagnostic: each step prints as it ends)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))
import torch  # noqa: E402
import bihrt  # noqa: E402

t = time.time()
tris = bihrt.scenes.soup(1_000_000, seed=1)
d = torch.from_numpy(tris).cuda()
g = bihrt.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0])
print("build", time.time() - t, flush=True)
w, h = int(sys.argv[1]), int(sys.argv[2])
for k in range(2):
    t = time.time()
    out = torch.zeros(h * w, dtype=torch.int32, device="cuda")
    hits = torch.zeros(h * w * 4, dtype=torch.int32, device="cuda")
    r = bihrt.Renderer(g, w, h, spp=4)
    r.render_whitted_device(out.data_ptr(), 0, hits_ptr=hits.data_ptr())
    print("issued", time.time() - t, flush=True)
    r.sync()
    print("whitted", w, h, time.time() - t, int(hits.sum()), flush=True)
