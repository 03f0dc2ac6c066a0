"""Diagnostic for test_bins_list_total_past_u32_renders_without_bins."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))
import torch  # noqa: E402
import bihrt  # noqa: E402
from bihrt.tiling import band_rows  # noqa: E402
w, h = 1920, 1080
cam = np.array(bihrt.camera_reference(w, h).as_list(), np.float32)
O, llc, hh, vv = cam[0:3], cam[3:6], cam[6:9], cam[9:12]
for n in (int(sys.argv[1]),):
    d = (1.2 + 1e-5 * np.arange(n, dtype=np.float64))[:, None]
    P = lambda u, v: O[None, :] + d * ((llc + u * hh + v * vv) - O)[None, :]
    tris = np.concatenate([P(-20, -20), P(-20, 40), P(40, -20)], 1).astype(np.float32)   # front-facing
    g = bihrt.GPUArrayManager(tris)
    print("n", n, "U", g.info().n_unique, flush=True)
    rows = band_rows(h, 4, 67, 270)
    for trav in (bihrt.TRAVERSE_ANYHIT, bihrt.TRAVERSE_REFERENCE):
        out = torch.zeros(rows.nrows * w, dtype=torch.int32, device="cuda")
        r = bihrt.Renderer(g, w, h)
        r.render_device(out.data_ptr(), 0, rows=rows, traverse=trav)
        r.sync()
        a = out.cpu().numpy().view(np.uint32)
        st = g.bins_stats()
        print("trav", trav, "unique px", np.unique(a)[:5], "usable", st.usable, "entries", st.list_entries,
              "global", st.global_entries, "tiles", st.tiles_x, st.tiles_y, flush=True)
