set -u
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04m_tests.log 2>&1 || { tail -40 gpurun_out/r04m_tests.log; exit 1; }
tail -2 gpurun_out/r04m_tests.log
bash tools/gpu_habn.sh r04m 2 nohint base
