#!/usr/bin/env python3
"""Per-dispatch PMC values from rocprofv3 counter_collection.csv files:
prints, for every dispatch of kernels matching --kernel, its order, name
and each counter (summed over the dimensions rocprofv3 splits it into),
then the mean per kernel instance.  FETCH_SIZE is reported x2 (gfx950
correction, MI355X_MICROARCH.md) in MB next to the raw KB.
usage: pmc_dispatch.py DIR [--kernel k_render_bins]"""
import argparse
import collections
import csv
import glob
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="k_render_bins")
    a = ap.parse_args()
    vals = collections.OrderedDict()   # dispatch id -> {name, counters}
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"]
            if a.kernel not in name:
                continue
            did = int(row.get("Dispatch_Id") or row.get("Correlation_Id") or 0)
            m = re.search(r"(k_\w+<[^>]*>|k_\w+)", name)
            d = vals.setdefault(did, {"name": m.group(1) if m else name[:40], "c": collections.defaultdict(float)})
            d["c"][row["Counter_Name"]] += float(row["Counter_Value"])
    by = collections.defaultdict(list)
    for k, (did, d) in enumerate(sorted(vals.items())):
        parts = []
        for c, v in sorted(d["c"].items()):
            if c == "FETCH_SIZE":
                parts.append("FETCH_SIZE %.0f KB (x2 = %.1f MB)" % (v, 2 * v / 1024))
            elif c == "WRITE_SIZE":
                parts.append("WRITE_SIZE %.1f MB" % (v / 1024))
            else:
                parts.append("%s %.4g" % (c, v))
        print("%3d dispatch %6d %-24s %s" % (k, did, d["name"], "  ".join(parts)))
        by[d["name"]].append(d["c"])
    for name, rows in by.items():
        keys = sorted(rows[0])
        print("mean over %d x %s: %s" % (len(rows), name, "  ".join(
            "%s %.4g" % (c, sum(r[c] for r in rows) / len(rows)) for c in keys)))


if __name__ == "__main__":
    main()
