# Round 5: the driver's command after the traffic probe's shape change, and
# per-dispatch PMC of the roofline samples' shape (16-frame calls rotating
# over 3 streams, each synchronised: ring instance, shared grid).
set -u
T=${1:-r05y}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u bench.py > $O/bench_final.json 2> $O/bench_final.err || { tail -30 $O/bench_final.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('head %.5f ms/frame %.1f G' % (d['ms_per_step'], d['value']/1e9), 'launch %.4f' % d['roofline']['launch_ms'], 'frac', d['roofline']['frac'], 'traffic', d['roofline']['traffic'])
" $O/bench_final.json
cd /tmp && export TMPDIR=/tmp
pmc() {   # pmc NAME COUNTERS
  local N=$1; local C=$2
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/$N -o pmc --output-format csv -- \
      python3 $R/tools/call_breakdown.py --frames 16 --calls 8 --warm 4 --sync 1 --streams 3 > $O/$N.log 2>&1 || { tail -5 $O/$N.log; return 1; }
  python3 $R/tools/pmc_dispatch.py $O/$N > $O/${N}.txt; tail -2 $O/${N}.txt
}
pmc fetch_rot FETCH_SIZE &&
pmc write_rot WRITE_SIZE &&
pmc sq_rot "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES"
