#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line (round 6 fields)."""
import json
import sys

p = json.load(open(sys.argv[1]))
if "parsed" in p:
    p = p["parsed"]
rf = p["roofline"]
print(f"headline {p['value'] / 1e9:.1f} G rays/s  {p['ms_per_step']:.4f} ms/frame  timed_outputs_equal "
      f"{p.get('timed_outputs_equal')}  frac {rf['frac']:.3f} (isolated {rf.get('frac_isolated_launches') or 0:.3f})")
w = rf.get("window") or {}
if w:
    print(f"  window kernel {w['kernel_ms_per_frame']:.4f} ms/frame, replica {w['ms_per_step']:.4f}")
iss = rf.get("issue") or {}
if iss:
    print(f"  VALU {iss['valu_per_frame'] / 1e6:.2f} M/frame SALU {iss['salu_per_frame'] / 1e6:.2f} M  issue frac "
          f"{iss['valu_issue_frac']:.3f}")
for k in ("one_in_flight", "with_rebuild", "dynamic_rebuild", "moving_camera"):
    if p.get(k):
        print(f"{k:16s} {p[k]['ms_per_step']:.4f} ms/step")
h = p.get("host_loop")
if h:
    print("host_loop " + " ".join(f"{k} {v['ms_per_step']:.3f}" for k, v in h.items() if isinstance(v, dict)))
if p.get("band_share"):
    print(f"band_share {p['band_share']['projected_efficiency']:.3f}  full {p['band_share']['full_frame_ms_per_step']:.4f}"
          f" max share {max(p['band_share']['share_ms_per_step']):.4f}")
c5 = p.get("c5_10m_4k")
if c5:
    print(f"C5 {c5['ms_per_step']:.4f} ms/frame, band_share {(c5.get('band_share') or {}).get('projected_efficiency')}")
if p.get("c2_torus"):
    print(f"C2 {p['c2_torus']['ms_per_step']:.4f}")
if p.get("whitted_c4"):
    print(f"C4 {p['whitted_c4']['ms_per_frame']:.1f} ms/frame")
bad = [c for c in (p.get("timed_outputs") or {}).get("checks", []) if not c["equal"]]
if bad:
    print("UNEQUAL:", bad)
