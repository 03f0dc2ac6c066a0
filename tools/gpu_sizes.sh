# per-frame time vs image size (1M soup): fixed vs per-ray cost
set -u
for S in "64 64" "960 540" "1920 1080" "3840 2160"; do
  set -- $S
  timeout -k 10 200 python bench.py --width $1 --height $2 --steps 60 --warmup 10 --traffic 0 --cpu-baseline 0 --headline-only --kernel-samples 10 > gpurun_out/sz_$1.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/sz_$1.json').read().strip().splitlines()[-1]);print('$1x$2', 'inflight_ms', round(d['ms_per_step'],4), 'kernel_ms', round(d['roofline']['launch_ms'],4), 'Grays', round(d['value']/1e9,2))"
done
