# Round 5 final evidence: tests, the driver's command, its kernel stats,
# isolated ring 16-frame launches (per dispatch), per-dispatch PMC, windows.
set -u
T=${1:-r05y}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --durations=5 --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('head %.5f ms/frame %.1f G' % (d['ms_per_step'], d['value']/1e9), 'launch %.4f' % d['roofline']['launch_ms'], 'frac', d['roofline']['frac'])
" $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o k --output-format csv -- \
    python3 $R/bench.py --traffic 0 > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
BIH_STAMPED=0 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/g16_ring -o k --output-format csv -- \
    python3 $R/tools/call_breakdown.py --frames 16 --calls 20 --sync 1 > $O/g16_ring.log 2>&1 || exit 1
python3 $R/tools/call_timeline.py $O/g16_ring/k_kernel_trace.csv --show 1 --dispatch-csv $O/g16_ring_dispatches.csv > $O/g16_ring_timeline.txt
tail -8 $O/g16_ring_timeline.txt
pmc() {   # pmc NAME ENV COUNTERS
  local N=$1; local E=$2; local C=$3
  env $E timeout -s KILL 120 rocprofv3 --pmc $C -d $O/$N -o pmc --output-format csv -- \
      python3 $R/tools/call_breakdown.py --frames 16 --calls 8 --warm 4 --sync 1 > $O/$N.log 2>&1 || { tail -5 $O/$N.log; return 1; }
  python3 $R/tools/pmc_dispatch.py $O/$N > $O/${N}.txt; tail -2 $O/${N}.txt
}
pmc fetch_ring BIH_STAMPED=0 FETCH_SIZE &&
pmc write_ring BIH_STAMPED=0 WRITE_SIZE &&
pmc sq_ring BIH_STAMPED=0 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" || exit 1
win() {   # win NAME TOOL ARGS...
  local N=$1; local P=$2; shift 2
  timeout -k 10 180 rocprofv3 --kernel-trace -d $O/$N -o k --output-format csv -- \
      python3 $R/tools/$P "$@" > $O/$N.log 2>&1 || { tail -20 $O/$N.log; return 1; }
  python3 $R/tools/window_timeline.py $O/$N/k_kernel_trace.csv $O/$N.log > $O/${N}_timeline.txt
}
win full window_trace.py --repeat 3 &&
win share0 window_trace.py --share 0/8 --repeat 3 &&
win cam cam_window.py --repeat 2 && tail -9 $O/full_timeline.txt
