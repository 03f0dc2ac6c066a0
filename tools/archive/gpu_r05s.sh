# Round 5: the driver's command (bench.py defaults) and its kernel trace /
# stats (traffic passes off under the tracer), for profiles/r05.
set -u
T=${1:-r05s}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -c 1200 $O/bench.json; echo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o k --output-format csv -- \
    python3 $R/bench.py --traffic 0 > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
python3 -c "
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print('%-60s %6s %12.1f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
" $O/prof/k_kernel_stats.csv
