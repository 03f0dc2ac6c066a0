#!/bin/bash
# with_rebuild window traces (graph build vs launch by launch), round 6.
# usage: tools/gpu_rb_trace.sh <tag>   (on the GPU box)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
OUT=$R/gpurun_out/rb_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for g in 1 0; do
  BIH_BUILD_GRAPH=$g timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/g$g" -o rb --output-format csv -- \
      python3 "$R/tools/rb_window.py" --steps 20 --repeat 3 > "$OUT/g$g.log" 2>&1 || exit 1
  f=$(find "$OUT/g$g" -name "*kernel_trace.csv" | head -1)
  python3 "$R/tools/window_timeline.py" "$f" "$OUT/g$g.log" > "$OUT/timeline_g$g.txt" || exit 1
  s=$(find "$OUT/g$g" -name "*kernel_stats.csv" | head -1)
  cp "$s" "$OUT/stats_g$g.csv"
done
echo done
