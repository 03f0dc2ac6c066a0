# Round 5: fused XORWOW advance -- GPU tests, A/B vs the previous revision
# (driver command + per-call kernel traces), item timelines.
set -u
T=${1:-r05c}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
V=$R/bih-gpu-raytracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --durations=12 --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
grep -E "passed|failed|s call" $O/pytest.log | tail -16
for k in 1 2; do
  for X in work prev; do
    if [ $X = work ]; then L=""; else L=$V/libbih_amd_prev.so; fi
    BIH_LIB=$L timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --c5 0 --whitted-frames 0 \
        --cpu-baseline 0 --traffic 0 --no-reference-leg > $O/bench_${X}_$k.json 2> $O/bench_${X}_$k.err || { tail -20 $O/bench_${X}_$k.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'head %.4f' % d['ms_per_step'], 'launch %.4f' % (d['roofline']['launch_ms']/16), 'one %.4f' % d['one_in_flight']['ms_per_step'], 'cam %.4f' % d['moving_camera']['ms_per_step'], 'rb %.4f' % d['with_rebuild']['ms_per_step'], 'share %.3f' % d['band_share']['projected_efficiency'], 'c2 %.4f' % d['c2_torus']['ms_per_step'])
" $O/bench_${X}_$k.json $X | tee -a $O/ab.txt
  done
done
cd /tmp && export TMPDIR=/tmp
trace() {   # trace NAME LIB ARGS...
  local N=$1; local L=$2; shift 2
  BIH_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/$N -o k --output-format csv -- \
      python3 $R/tools/call_breakdown.py "$@" > $O/$N.log 2>&1 || { tail -20 $O/$N.log; return 1; }
  grep "^calls" $O/$N.log
  python3 $R/tools/call_timeline.py $O/$N/k_kernel_trace.csv --show 1 --dispatch-csv $O/${N}_dispatches.csv > $O/${N}_timeline.txt; tail -8 $O/${N}_timeline.txt
}
trace one_sync_work "" --frames 1 --calls 60 --sync 1 &&
trace g16_sync_work "" --frames 16 --calls 20 --sync 1 &&
trace g20_sync_work "" --frames 20 --calls 16 --sync 1 || exit 1
cd $R
tl() {   # tl NAME ARGS...
  local N=$1; shift
  rm -f $O/$N.bin
  BIH_LIB=$V/libbih_amd_tl.so BIH_TIMELINE_OUT=$O/$N.bin timeout -k 10 120 python3 tools/call_breakdown.py "$@" > $O/$N.log 2>&1 || { tail -20 $O/$N.log; return 1; }
  grep "^calls" $O/$N.log
  python3 tools/bins_timeline.py $O/$N.bin --skip 4 --show 2 > $O/${N}_tl.txt; tail -30 $O/${N}_tl.txt
}
tl tl_one --frames 1 --calls 24 --warm 4 &&
tl tl_g16 --frames 16 --calls 8 --warm 4 &&
tl tl_share8_g16 --frames 16 --calls 8 --warm 4 --share 0/8
