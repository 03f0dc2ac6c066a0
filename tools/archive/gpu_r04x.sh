set -u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "bin or camera or render or headline" > gpurun_out/r04x_tests.log 2>&1 || { tail -40 gpurun_out/r04x_tests.log; exit 1; }
tail -1 gpurun_out/r04x_tests.log
bash tools/gpu_kcam_ab.sh r04y notab tabw6 nosplit
