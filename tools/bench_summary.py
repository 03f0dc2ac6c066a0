#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line (the file holds one line)."""
import json
import sys

d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
rf = d.get("roofline") or {}
print("value %.4g rays/s  ms/step %.4f  n_gpus %s  scaling %s" % (d["value"], d["ms_per_step"], d["n_gpus"],
                                                                  d["scaling"]))
print("roofline frac %s  frac_algorithmic %s  launch_ms %s" % (rf.get("frac"), rf.get("frac_algorithmic"),
                                                               rf.get("launch_ms")))
print("allocs in headline", d.get("device_allocs_in_headline"), "world", d.get("world_size"), d.get("backend"),
      d.get("rccl_version"), "frac_compulsory", rf.get("frac_compulsory"))
for k in ("one_in_flight", "moving_camera", "with_rebuild", "other_traversal", "band_share",
          "other_decomposition", "whitted_c4", "c2_torus", "c5_10m_4k"):
    v = d.get(k)
    if v:
        print(k, {kk: v[kk] for kk in v if kk in ("value", "ms_per_step", "projected_efficiency",
                                                  "share_ms_per_step", "build_ms", "kernel_ms",
                                                  "ms_per_frame", "rays_traced_per_s", "rebuild_ms")})
c = d.get("cpu_baseline")
if c:
    print("cpu", c["value"], c["cores"], c.get("cpu_model"), c.get("affinity_cpus"))
    for k, v in (c.get("legs") or {}).items():
        print("  cpu leg", k, "%.4g rays/s" % v["value"], v["cores"], "thr", "%.1fs" % v["seconds"])
print("parity_sample_rows_equal", d.get("parity_sample_rows_equal"))
