#!/usr/bin/env python3
"""Per-call kernel timeline of tools/prof_share.py traces: per kernel name the
mean duration over the last calls, and the mean span from a call's first
kernel start to its last kernel end (the call's device time)."""
import csv
import re
import sys


def main():
    for path in sys.argv[1:]:
        rows = list(csv.DictReader(open(path)))
        ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
        # the last 30 calls: k_rng_advance starts each call
        starts = [i for i, e in enumerate(ev) if "k_rng_advance" in e[2]]
        calls = []
        for a, b in zip(starts, starts[1:] + [len(ev)]):
            calls.append(ev[a:b])
        calls = calls[-30:]
        dur = {}
        for c in calls:
            for s, e, n in c:
                m = re.search(r"(k_\w+)", n)
                key = m.group(1) if m else n[:40]
                dur.setdefault(key, []).append((e - s) / 1e3)
        print(path)
        for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
            print(f"  {k:42s} n={len(v):3d} mean {sum(v)/len(v):8.2f} us")
        gaps = [(c[1][0] - c[0][1]) / 1e3 for c in calls if len(c) > 1]
        spans = [(max(e for _, e, _ in c) - c[0][0]) / 1e3 for c in calls]
        firsts = [c[0][0] for c in calls]
        per = [(b - a) / 1e3 for a, b in zip(firsts, firsts[1:])]
        print(f"  call span mean {sum(spans)/len(spans):.2f} us; call-to-call start {sum(per)/max(1,len(per)):.2f} us;"
              f" advance->render gap {sum(gaps)/max(1,len(gaps)):.2f} us")


if __name__ == "__main__":
    main()
