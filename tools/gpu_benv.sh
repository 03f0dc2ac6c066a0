# bench headline (in flight) and isolated render timing under env settings
set -u
T=$1; shift
for E in "" "$@"; do
  env $E timeout -k 10 120 python tools/time_render.py --tag x > gpurun_out/${T}.time 2>/dev/null || exit 1
  env $E timeout -k 10 200 python bench.py --traffic 0 --cpu-baseline 0 --headline-only --kernel-samples 0 --steps 2000 --warmup 200 > gpurun_out/${T}.json 2>/dev/null || exit 1
  python3 -c "import json,sys;t=json.loads(open(sys.argv[1]).read());b=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]);print(sys.argv[3], 'iso', round(t['ms_mean'],4), 'inflight', round(b['ms_per_step'],4), 'Grays', round(b['value']/1e9,2))" gpurun_out/${T}.time gpurun_out/${T}.json "[$E]"
done
