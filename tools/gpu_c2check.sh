timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -k "c2_torus or pair_results" > gpurun_out/r03s2k_tests.log 2>&1; tail -4 gpurun_out/r03s2k_tests.log
timeout -k 10 300 python bench.py --steps 256 --warmup 32 --traffic 0 --cpu-baseline 0 --whitted-frames 0 --no-reference-leg --no-rebuild-leg > gpurun_out/r03s2k_bench.json 2>gpurun_out/r03s2k_bench.err || { tail -5 gpurun_out/r03s2k_bench.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/r03s2k_bench.json').read().strip().splitlines()[-1]);print(d['value'], d['c2_torus'])"
