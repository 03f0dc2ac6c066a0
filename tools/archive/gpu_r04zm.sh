set -u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "rebuild or static or render_matches or frames" > gpurun_out/r04zm_tests.log 2>&1 || { tail -40 gpurun_out/r04zm_tests.log; exit 1; }
tail -1 gpurun_out/r04zm_tests.log
bash tools/gpu_benv_quick.sh r04zm 2 noprio
