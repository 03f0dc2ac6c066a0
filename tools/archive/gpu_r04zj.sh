set -u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "render or rebuild or frames or camera or bin" > gpurun_out/r04zj_tests.log 2>&1 || { tail -40 gpurun_out/r04zj_tests.log; exit 1; }
tail -1 gpurun_out/r04zj_tests.log
bash tools/gpu_benv_quick.sh r04zj 2 nofuse
