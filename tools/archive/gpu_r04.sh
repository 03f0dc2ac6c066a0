# Round-4 GPU check: selected (or all) gpu tests, the driver's bench command,
# a kernel-trace profile of the headline.
# usage: bash tools/gpu_r04.sh TAG "PYTEST -k EXPR or ''" [bench args...]
set -u
T=$1; K=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KA[@]}" \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 900 python bench.py "$@" > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/${T}_bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --headline-only --steps 20 --warmup 5 --traffic 0 --cpu-baseline 0 --c5 0 \
  > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/${T}_kernel_stats.csv
head -12 gpurun_out/${T}_kernel_stats.csv | cut -c1-160
tail -1 gpurun_out/${T}_prof.log | cut -c1-400
