#!/usr/bin/env python3
"""Splits a rocprofv3 kernel trace (kernel_trace.csv) of tools/call_breakdown.py
into render calls -- a call starts at a k_rng_advance dispatch -- and prints,
per call, each kernel's start (relative to the call's first dispatch) and
duration, then the mean over the calls (second half, warm) of: advance,
advance->render gap, render, render->fallback gap, fallback, call span, and the
start-to-start period.  Also writes the per-dispatch k_render_bins durations
(`--dispatch-csv`), the evidence a launch_ms figure can be recomputed from.
usage: tools/call_timeline.py kernel_trace.csv [--show N] [--dispatch-csv out.csv]"""
import argparse
import csv
import re


def name(r):
    m = re.search(r"(k_\w+|__amd\w+|\w*elementwise\w*)", r["Kernel_Name"])
    return m.group(1) if m else r["Kernel_Name"][:24]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--show", type=int, default=3)
    ap.add_argument("--dispatch-csv", default="")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    # a call starts at its k_rng_advance, or at its k_render_bins when the
    # render advances the XORWOW state itself (no advance launch)
    calls, cur = [], None
    for r in rows:
        n = name(r)
        if n == "k_rng_advance" or (n == "k_render_bins" and (cur is None or any(x[0] == n for x in cur))):
            cur = []
            calls.append(cur)
        if cur is not None:
            cur.append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r))
    calls = [c for c in calls if any(n == "k_render_bins" for n, *_ in c)]
    if not calls:
        print("no render calls found")
        return
    for c in calls[-a.show:]:
        t0 = c[0][1]
        print("---")
        for n, s, e, _ in c:
            print("  %-20s start %8.2f dur %8.2f us" % (n, (s - t0) / 1e3, (e - s) / 1e3))
    half = calls[len(calls) // 2:]
    acc = {}

    def add(k, v):
        acc.setdefault(k, []).append(v)

    for i, c in enumerate(half):
        d = {n: (s, e) for n, s, e, _ in c}
        if not all(k in d for k in ("k_render_bins", "k_render_fallback")):
            continue
        ren, fb = d["k_render_bins"], d["k_render_fallback"]
        if "k_rng_advance" in d:
            adv = d["k_rng_advance"]
            add("advance", adv[1] - adv[0])
            add("gap advance->render", ren[0] - adv[1])
        add("render", ren[1] - ren[0])
        add("gap render->fallback", fb[0] - ren[1])
        add("fallback", fb[1] - fb[0])
        add("span first start->last end", c[-1][2] - c[0][1])
        if i + 1 < len(half):
            add("period start->next start", half[i + 1][0][1] - c[0][1])
    print("calls %d (mean over the last %d):" % (len(calls), len(half)))
    for k, v in acc.items():
        v = sorted(v)
        print("  %-28s mean %8.2f  median %8.2f  min %8.2f  max %8.2f us" %
              (k, sum(v) / len(v) / 1e3, v[len(v) // 2] / 1e3, v[0] / 1e3, v[-1] / 1e3))
    if a.dispatch_csv:
        with open(a.dispatch_csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["call", "kernel", "start_ns_rel", "duration_ns", "grid", "workgroup"])
            for i, c in enumerate(calls):
                t0 = c[0][1]
                for n, s, e, r in c:
                    w.writerow([i, n, s - t0, e - s, r.get("Grid_Size", r.get("Grid_Size_X", "")),
                                r.get("Workgroup_Size", r.get("Workgroup_Size_X", ""))])


if __name__ == "__main__":
    main()
