timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02c_tests.log 2>&1; rc=$?; tail -5 gpurun_out/r02c_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/time_render.py --tag bins > gpurun_out/r02c_time.jsonl 2>&1 || exit 1
BIH_BINS=0 timeout -k 10 120 python tools/time_render.py --tag nobins >> gpurun_out/r02c_time.jsonl 2>&1 || exit 1
cut -c1-300 gpurun_out/r02c_time.jsonl
timeout -k 10 300 python bench.py --traffic 0 --cpu-baseline 0 --headline-only > gpurun_out/r02c_bench.json 2>&1; echo bench=$?; cut -c1-400 gpurun_out/r02c_bench.json
