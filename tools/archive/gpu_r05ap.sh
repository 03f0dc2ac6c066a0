# Round 5: the round-end sequence rehearsed on the final tree: GPU suite,
# smoke(), the driver's command.
set -u
T=${1:-r05ap}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('head %.5f ms/frame %.1f G' % (d['ms_per_step'], d['value']/1e9), 'frac', round(d['roofline']['frac'],3), 'one', round(d['one_in_flight']['ms_per_step'],4), 'share', round(d['band_share']['projected_efficiency'],3))
" $O/bench.json
