set -u
for V in tab; do
  BIH_LIB=$GRAFT_REPO_ROOT/bih-gpu-raytracer_amd/lib/variants/libbih_amd_$V.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "bin or camera" > gpurun_out/r04y_tests_$V.log 2>&1 || { tail -40 gpurun_out/r04y_tests_$V.log; exit 1; }
  tail -1 gpurun_out/r04y_tests_$V.log
done
bash tools/gpu_kcam_ab.sh r04y tab notab tabw6
bash tools/gpu_wh_ab.sh r04y whs2 whs8
