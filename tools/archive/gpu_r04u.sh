set -u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "rebuild or render or headline or band or frames or camera" > gpurun_out/r04u_tests.log 2>&1 || { tail -40 gpurun_out/r04u_tests.log; exit 1; }
tail -1 gpurun_out/r04u_tests.log
for s in 1 0; do timeout -k 10 300 python tools/time_host_rebuild.py --static $s || exit 1; done
timeout -k 10 600 python bench.py --no-reference-leg --c5 0 --whitted-frames 0 --cpu-baseline 0 --traffic 0 > gpurun_out/r04u_bench.json 2> gpurun_out/r04u_bench.err || { tail -30 gpurun_out/r04u_bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/r04u_bench.json
