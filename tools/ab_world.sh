# per-GPU share of a W-GPU frame on one GPU (strong-scaling estimate)
set -u
TAG=$1
J=gpurun_out/abw_$TAG.jsonl; rm -f $J
for W in 1 2 4 8; do
  timeout -k 10 120 python tools/time_render.py --traverse anyhit --frames 20 --world $W --tag w$W >> $J 2>>gpurun_out/abw_$TAG.err || { echo "fail $W"; exit 1; }
done
python3 -c "
import json
rows=[json.loads(l) for l in open('$J')]
t1=rows[0]['ms_median']
for r in rows: print(r['world'], round(r['ms_median'],3), 'eff', round(t1/(r['world']*r['ms_median']),3))"
