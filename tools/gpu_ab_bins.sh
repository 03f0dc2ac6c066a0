# tests, timing (bins on / off), counters variant
set -u
T=$1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -5 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/time_render.py --tag bins > gpurun_out/${T}_time.jsonl 2>&1 || exit 1
BIH_BINS=0 timeout -k 10 120 python tools/time_render.py --tag nobins >> gpurun_out/${T}_time.jsonl 2>&1 || exit 1
grep -o '"tag[^,]*\|"ms_mean[^,]*\|"img_hash[^,}]*' gpurun_out/${T}_time.jsonl
BIH_LIB=bih-gpu-raytracer_amd/lib/variants/libbih_amd_fc.so timeout -k 10 120 python tools/fast_counters.py --frames 2 > gpurun_out/${T}_fc.log 2>&1 || exit 1
grep bin-counters gpurun_out/${T}_fc.log
timeout -k 10 300 python bench.py --traffic 0 --cpu-baseline 0 --headline-only > gpurun_out/${T}_bench.json 2>&1; echo bench=$?; grep -o '"value[^,]*\|"ms_per_step[^,]*' gpurun_out/${T}_bench.json
