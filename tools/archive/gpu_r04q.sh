set -u
timeout -k 10 300 python -u -m pytest tests/test_whitted.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04q_tests.log 2>&1 || { tail -30 gpurun_out/r04q_tests.log; exit 1; }
tail -1 gpurun_out/r04q_tests.log
bash tools/gpu_wh_ab.sh r04q whnp whold || exit 1
bash tools/gpu_rebuild_prof.sh r04q
