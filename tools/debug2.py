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
viol = s[:, 2] >= 1000000
print("violating rays", viol.sum(), "first-step values", np.unique(s[viol, 2] - 1000000)[:20])
bad = np.nonzero(s[:, 0] != rs[:, 0])[0]
print("mismatch", bad.size, "of which flagged", viol[bad].sum())
