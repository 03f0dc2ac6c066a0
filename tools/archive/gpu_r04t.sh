set -u
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04t_tests.log 2>&1 || { tail -40 gpurun_out/r04t_tests.log; exit 1; }
tail -1 gpurun_out/r04t_tests.log
timeout -k 10 300 python tools/time_host_rebuild.py > gpurun_out/r04t_host.txt 2>&1 || { tail -5 gpurun_out/r04t_host.txt; exit 1; }
cat gpurun_out/r04t_host.txt
timeout -k 10 900 python bench.py > gpurun_out/r04t_bench.json 2> gpurun_out/r04t_bench.err || { tail -30 gpurun_out/r04t_bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/r04t_bench.json
bash tools/gpu_rebuild_prof.sh r04t 2>&1 | tail -16
