# Round 5: static queue rounds in one-frame launches -- tests, A/B of the round count,
# stamped state off; traces.
set -u
T=${1:-r05n}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --durations=5 --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab5.sh $T 2 base base+BIH_STATIC_ROUNDS=1 base+BIH_STATIC_ROUNDS=2 base+BIH_STATIC_ROUNDS=5 base+BIH_STAMPED=0 || exit 1
cd /tmp && export TMPDIR=/tmp
trace() {   # trace NAME ARGS...
  local N=$1; shift
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/$N -o k --output-format csv -- \
      python3 $R/tools/call_breakdown.py "$@" > $O/$N.log 2>&1 || { tail -20 $O/$N.log; return 1; }
  grep "^calls" $O/$N.log
  python3 $R/tools/call_timeline.py $O/$N/k_kernel_trace.csv --show 1 --dispatch-csv $O/${N}_dispatches.csv > $O/${N}_timeline.txt; tail -8 $O/${N}_timeline.txt
}
trace g16_sync --frames 16 --calls 20 --sync 1 &&
trace one_sync --frames 1 --calls 60 --sync 1
