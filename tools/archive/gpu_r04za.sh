set -u
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04za_tests.log 2>&1 || { tail -40 gpurun_out/r04za_tests.log; exit 1; }
tail -1 gpurun_out/r04za_tests.log
bash tools/gpu_wh_ab.sh r04za whs32 || exit 1
timeout -k 10 900 python bench.py > gpurun_out/r04za_bench.json 2> gpurun_out/r04za_bench.err || { tail -30 gpurun_out/r04za_bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/r04za_bench.json
bash tools/gpu_kcam.sh r04za
