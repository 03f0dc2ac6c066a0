#!/usr/bin/env python3
"""Kernels of a rocprofv3 kernel trace inside the host windows printed by
tools/window_trace.py: per window, each kernel's start / end relative to the
window's start (us), and the host's issue times.
usage: window_timeline.py KERNEL_TRACE.csv WINDOW_TRACE.log"""
import csv
import re
import sys


def main():
    quiet = "--quiet" in sys.argv
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    for line in open(sys.argv[2]):
        if not line.startswith("window"):
            continue
        tok = line.split()
        t0 = int(tok[tok.index("start_ns") + 1])
        t1 = int(tok[tok.index("end_ns") + 1])
        issued = [int(x) for x in tok[tok.index("issued_ns") + 1: tok.index("end_ns")]]
        print(line.strip())
        print("  host issue done at: " + ", ".join("%.1f" % ((x - t0) / 1e3) for x in issued) + " us")
        for r in rows:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if e < t0 or s > t1:
                continue
            m = re.search(r"(k_\w+(?:<[^>]*>)?|__amd\w+)", r["Kernel_Name"])
            nm = m.group(1) if m else r["Kernel_Name"][:30]
            if not quiet:
                print("  %-28s q%-3s start %8.1f end %8.1f dur %7.1f" % (nm, r.get("Queue_Id", "?"), (s - t0) / 1e3,
                                                                      (e - t0) / 1e3, (e - s) / 1e3))
        print("  window end %.1f us" % ((t1 - t0) / 1e3))
        # per kernel: launches and device time inside the window
        agg = {}
        for r in rows:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if e < t0 or s > t1:
                continue
            m = re.search(r"(k_\w+(?:<[^>]*>)?|__amd\w+)", r["Kernel_Name"])
            nm = m.group(1) if m else r["Kernel_Name"][:30]
            n, tot = agg.get(nm, (0, 0))
            agg[nm] = (n + 1, tot + e - s)
        for nm, (n, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print("  sum %-28s %4d x %8.1f us = %9.1f us" % (nm, n, tot / n / 1e3, tot / 1e3))


if __name__ == "__main__":
    main()
