# Round 5, first GPU call: tests, the driver's bench command, and kernel
# traces of the per-call shapes (tools/call_breakdown.py + call_timeline.py).
# usage: bash tools/gpu_r05a.sh TAG
set -u
T=${1:-r05a}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
python3 tools/bench_summary.py $O/bench_driver.json 2>/dev/null | head -30 || true
cd /tmp && export TMPDIR=/tmp
trace() {   # trace NAME ARGS...
  local N=$1; shift
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/$N -o k --output-format csv -- \
      python3 $R/tools/call_breakdown.py "$@" > $O/$N.log 2>&1 || { tail -20 $O/$N.log; return 1; }
  grep calls $O/$N.log
  python3 $R/tools/call_timeline.py $(ls $O/$N/*/k_kernel_trace.csv $O/$N/k_kernel_trace.csv 2>/dev/null | head -1) \
      --show 1 --dispatch-csv $O/${N}_dispatches.csv > $O/${N}_timeline.txt && tail -9 $O/${N}_timeline.txt
}
trace one_sync --frames 1 --calls 60 --sync 1 &&
trace g16_sync --frames 16 --calls 20 --sync 1 &&
trace share8_g16_sync --frames 16 --calls 20 --sync 1 --share 0/8 &&
trace share8_g1_sync --frames 1 --calls 40 --sync 1 --share 0/8 &&
trace g16_flight3 --frames 16 --calls 30 --sync 0 --streams 3 &&
trace one_flight3 --frames 1 --calls 90 --sync 0 --streams 3
