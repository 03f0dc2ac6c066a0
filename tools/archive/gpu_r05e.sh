# Round 5: cost-ordered queue with heavy-tile frame splitting -- tests, A/B
# (driver command), item timelines, kernel traces.
set -u
T=${1:-r05e}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
V=$R/bih-gpu-raytracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --durations=5 --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for k in 1 2; do
  for X in cost nocost; do
    L=""; E=1
    [ $X = prev ] && L=$V/libbih_amd_prev.so
    [ $X = nocost ] && E=0
    BIH_LIB=$L BIH_COST_QUEUE=$E timeout -k 10 300 python -u bench.py --c5 0 --whitted-frames 0 \
        --cpu-baseline 0 --traffic 0 --no-reference-leg > $O/bench_${X}_$k.json 2> $O/bench_${X}_$k.err || { tail -20 $O/bench_${X}_$k.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'head %.4f' % d['ms_per_step'], 'launch %.4f' % (d['roofline']['launch_ms']/16), 'one %.4f' % d['one_in_flight']['ms_per_step'], 'cam %.4f' % d['moving_camera']['ms_per_step'], 'rb %.4f' % d['with_rebuild']['ms_per_step'], 'share %.3f' % d['band_share']['projected_efficiency'], 'c2 %.4f' % d['c2_torus']['ms_per_step'])
" $O/bench_${X}_$k.json $X | tee -a $O/ab.txt
  done
done
BIH_COST_QUEUE=1 timeout -k 10 300 python -u bench.py --steps 500 --warmup 50 --c5 0 --whitted-frames 0 \
    --cpu-baseline 0 --traffic 0 --no-reference-leg --headline-only > $O/bench_cost_500.json 2> $O/bench_cost_500.err && \
    python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('cost 500 steps head %.4f' % d['ms_per_step'])" $O/bench_cost_500.json | tee -a $O/ab.txt
tl() {   # tl NAME COST ARGS...
  local N=$1; local C=$2; shift 2
  rm -f $O/$N.bin
  BIH_COST_QUEUE=$C BIH_LIB=$V/libbih_amd_tl.so BIH_TIMELINE_OUT=$O/$N.bin timeout -k 10 120 python3 tools/call_breakdown.py "$@" > $O/$N.log 2>&1 || { tail -20 $O/$N.log; return 1; }
  grep "^calls" $O/$N.log
  python3 tools/bins_timeline.py $O/$N.bin --skip 4 --show 1 > $O/${N}_tl.txt; tail -22 $O/${N}_tl.txt
}
tl tl_g16_cost 1 --frames 16 --calls 6 --warm 4 &&
tl tl_one_cost 1 --frames 1 --calls 16 --warm 4 || exit 1
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
