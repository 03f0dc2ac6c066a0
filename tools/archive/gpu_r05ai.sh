# Round 5: the 500-step steady state (--steps 500 --warmup 50; not the
# driver's command), headline only
set -u
T=${1:-r05ai}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
for k in 1 2; do
timeout -k 10 300 python -u bench.py --steps 500 --warmup 50 --headline-only --cpu-baseline 0 --traffic 0 \
    > $O/bench500_$k.json 2> $O/bench500_$k.err || { tail -20 $O/bench500_$k.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('500 steps %.5f ms/frame %.1f G' % (d['ms_per_step'], d['value']/1e9))" $O/bench500_$k.json
done
