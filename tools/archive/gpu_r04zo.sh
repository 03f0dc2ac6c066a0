set -u
BIH_LIB=$GRAFT_REPO_ROOT/bih-gpu-raytracer_amd/lib/variants/libbih_amd_sb5.so timeout -k 10 300 python -u -m pytest tests/test_whitted.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04zo_tests.log 2>&1 || { tail -30 gpurun_out/r04zo_tests.log; exit 1; }
tail -1 gpurun_out/r04zo_tests.log
bash tools/gpu_wh_ab.sh r04zo sb4 sb5 sb6
