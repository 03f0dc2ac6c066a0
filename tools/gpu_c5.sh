# config C5's scene on one GPU (10M tris, 3840x2160) + the empty frame.
# usage: bash tools/gpu_c5.sh TAG
set -u
T=${1:-c5}
timeout -k 10 300 python tools/time_empty.py > gpurun_out/${T}_empty.txt 2>&1 || exit 1
cat gpurun_out/${T}_empty.txt | tail -3
timeout -k 10 600 python -u bench.py --tris 10000000 --width 3840 --height 2160 --steps 96 --warmup 16 --traffic 0 --cpu-baseline 0 --no-reference-leg --whitted-frames 0 > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err || { tail -5 gpurun_out/${T}_c5.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/${T}_c5.json').read().strip().splitlines()[-1])
print({k:d[k] for k in ('value','ms_per_step','build_ms')}, 'bins', d.get('bins',{}).get('list_entries'), 'usable', d.get('bins',{}).get('usable'))
for k in ('one_in_flight','with_rebuild','moving_camera','band_share'): print(k, json.dumps(d.get(k))[:300])
"
