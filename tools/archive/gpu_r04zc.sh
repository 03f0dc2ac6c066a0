set -u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "render or headline or band or frames or camera or rebuild or bin" > gpurun_out/r04zc_tests.log 2>&1 || { tail -40 gpurun_out/r04zc_tests.log; exit 1; }
tail -1 gpurun_out/r04zc_tests.log
bash tools/gpu_benv_quick.sh r04zc 2 grab1 grab2 grab8
