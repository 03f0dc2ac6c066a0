set -u
BIH_LIB=$GRAFT_REPO_ROOT/bih-gpu-raytracer_amd/lib/variants/libbih_amd_fptab.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "bin or camera" > gpurun_out/r04z_tests.log 2>&1 || { tail -40 gpurun_out/r04z_tests.log; exit 1; }
tail -1 gpurun_out/r04z_tests.log
bash tools/gpu_kcam_ab.sh r04z fptab fptab5
bash tools/gpu_wh_ab.sh r04z whs16
