# GPU tests, render timing (bins on/off), bin counters, bench headline.
# usage: bash tools/gpu_quick.sh TAG
set -u
T=$1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit 1
J=gpurun_out/${T}_time.jsonl; rm -f $J
timeout -k 10 120 python tools/time_render.py --tag bins >> $J 2>/dev/null || exit 1
grep -o '"tag[^,]*\|"ms_mean[^,]*' $J
FC=bih-gpu-raytracer_amd/lib/variants/libbih_amd_fc.so
if [ -f $FC ]; then
  BIH_LIB=$FC timeout -k 10 120 python tools/fast_counters.py --frames 2 > gpurun_out/${T}_fc.log 2>&1 || exit 1
  grep bin-counters gpurun_out/${T}_fc.log | tail -1
fi
timeout -k 10 300 python bench.py --traffic 0 --cpu-baseline 0 --headline-only > gpurun_out/${T}_bench.json 2>&1 || exit 1
grep -o '"value[^,]*\|"ms_per_step[^,]*' gpurun_out/${T}_bench.json | head -2
