#!/usr/bin/env python3
"""Per-kernel averages of a tools/profile.sh output directory:
python tools/summarize_prof.py gpurun_out/prof_<tag> [kernel-substring]"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "k_render"
    for f in sorted(glob.glob(os.path.join(d, "*", "*kernel_stats.csv"))):
        for r in csv.DictReader(open(f)):
            if pat in r["Name"]:
                print(f"{r['Name'][:90]}: calls {r['Calls']} avg {float(r['AverageNs'])/1e6:.3f} ms "
                      f"min {float(r['MinNs'])/1e6:.3f} max {float(r['MaxNs'])/1e6:.3f}")
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(f"  {k:28s} n={len(v):3d} avg/launch {sum(v)/len(v):.6g}")


if __name__ == "__main__":
    main()
