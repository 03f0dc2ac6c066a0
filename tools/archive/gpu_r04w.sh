bash tools/gpu_kcam_ab.sh r04w fp1 fp2 fp4 fp8
