# tests, then render timing + bench headline for the default library and each variant
set -u
T=$1; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit 1
for V in default "$@"; do
  if [ "$V" = default ]; then L=""; else L=bih-gpu-raytracer_amd/lib/variants/libbih_amd_$V.so; fi
  BIH_LIB=$L timeout -k 10 120 python tools/time_render.py --tag $V > gpurun_out/${T}_$V.time 2>/dev/null || exit 1
  BIH_LIB=$L timeout -k 10 200 python bench.py --traffic 0 --cpu-baseline 0 --headline-only --kernel-samples 0 --steps 2000 --warmup 200 > gpurun_out/${T}_$V.json 2>/dev/null || exit 1
  python3 -c "import json,sys;t=json.loads(open(sys.argv[1]).read());b=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]);print(sys.argv[3], 'iso', round(t['ms_mean'],4), 'inflight', round(b['ms_per_step'],4), 'Grays', round(b['value']/1e9,2))" gpurun_out/${T}_$V.time gpurun_out/${T}_$V.json $V
done
