#!/bin/bash
# Builder kernels per library variant: rocprofv3 kernel stats of
# tools/build_loop.py (30 rebuilds of the 1M soup, nothing beside them).
# usage: tools/gpu_build_ab.sh TAG VARIANT...   (base = the in-tree library)
set -u
T=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
V=$R/bih-gpu-raytracer_amd/lib/variants
cd /tmp && export TMPDIR=/tmp
for X in "$@"; do
  L=""; [ $X != base ] && L=$V/libbih_amd_$X.so
  BIH_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$X -o bl --output-format csv -- \
      python3 $R/tools/build_loop.py > $O/$X.log 2>&1 || { tail -20 $O/$X.log; exit 1; }
  f=$(find $O/$X -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$X" <<'PY' | tee -a $O/summary.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = 0.0
out = []
for r in rows:
    import re
    m = re.search(r"(k_\w+|__amd\w+)", r["Name"])
    nm = m.group(1) if m else r["Name"][:20]
    if nm.startswith("__amd"):
        continue
    avg = float(r["AverageNs"]) / 1e3
    calls = int(r["Calls"])
    per_build = avg * calls / 32
    tot += per_build
    out.append("%s %.1f" % (nm, avg))
print(sys.argv[2], "per-build kernel sum %.1f us |" % tot, ", ".join(out))
PY
  grep rebuilds $O/$X.log
done
