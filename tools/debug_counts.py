import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np, torch, bihrt, oracle as O
tris = bihrt.scenes.torus()
g = bihrt.GPUArrayManager(tris); ot = O.OracleTree(tris)
w, h, spp = 96, 54, 4
out = torch.zeros(w*h, dtype=torch.int32, device="cuda"); st = torch.zeros(3*w*h*spp, dtype=torch.int32, device="cuda")
r = bihrt.Renderer(g, w, h, spp=spp)
r.render_device(out.data_ptr(), 0, traverse=bihrt.TRAVERSE_REFERENCE, stats_ptr=st.data_ptr()); r.sync()
s = st.cpu().numpy().view(np.uint32).reshape(-1, 3)
ref, _, rs = ot.render(w, h, spp=spp, mode=0, ray_stats=True)
for c in range(3):
    d = s[:, c].astype(np.int64) - rs[:, c].astype(np.int64)
    bad = np.nonzero(d)[0]
    print("counter", c, "mismatch rays", bad.size, "gpu-ref sum", d.sum(), "first", [(int(b), int(s[b, c]), int(rs[b, c])) for b in bad[:8]])
if os.environ.get("DBG"):
    v = s[:, 0]
    print("codes", np.unique(v, return_counts=True))
    ora = rs[:, 0] > 0
    print("oracle live", ora.sum(), "gpu live-bit", (v % 10 == 1).sum(), "gpu alive", ((v // 10) % 10 == 1).sum(),
          "both", ((v % 10 == 1) & ora).sum())
