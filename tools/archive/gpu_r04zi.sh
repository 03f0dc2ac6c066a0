set -u
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04zi_tests.log 2>&1 || { tail -40 gpurun_out/r04zi_tests.log; exit 1; }
tail -1 gpurun_out/r04zi_tests.log
bash tools/gpu_benv_quick.sh r04zi 2 nofuse
