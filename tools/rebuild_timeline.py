#!/usr/bin/env python3
"""Timeline of the with_rebuild leg from a rocprofv3 kernel trace of bench.py:
every kernel between consecutive k_prep launches (one rebuild + render step),
start relative to the step's k_prep, duration and queue; the mean step period.
usage: tools/rebuild_timeline.py kernel_trace.csv [steps to print]"""
import csv
import re
import sys


def name(r):
    m = re.search(r"(k_\w+|__amd\w+|\w*elementwise\w*)", r["Kernel_Name"])
    return m.group(1) if m else r["Kernel_Name"][:24]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    show = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    preps = [i for i, r in enumerate(rows) if name(r) == "k_prep"]
    # the with_rebuild leg: the longest run of k_prep launches each followed by a k_render_bins
    steps = []
    for a, b in zip(preps, preps[1:]):
        seg = rows[a:b]
        if any(name(r) == "k_render_bins" for r in seg):
            steps.append(seg)
    if not steps:
        print("no rebuild steps found")
        return
    for seg in steps[-show:]:
        t0 = int(seg[0]["Start_Timestamp"])
        print("---")
        for r in seg:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            print("  %-22s q%-3s start %8.1f dur %7.1f" % (name(r), r.get("Queue_Id", "?"), (s - t0) / 1e3,
                                                          (e - s) / 1e3))
    per = [(int(b[0]["Start_Timestamp"]) - int(a[0]["Start_Timestamp"])) / 1e3 for a, b in zip(steps, steps[1:])]
    per = per[len(per) // 2:]
    print("steps %d, k_prep-to-k_prep period (second half) mean %.1f us" % (len(steps), sum(per) / len(per)))
    busy = {}
    for seg in steps[len(steps) // 2:]:
        for r in seg:
            busy[name(r)] = busy.get(name(r), 0.0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    n = len(steps) - len(steps) // 2
    for k, v in sorted(busy.items(), key=lambda kv: -kv[1]):
        print("  %-22s %7.1f us per step" % (k, v / n))


if __name__ == "__main__":
    main()
