set -u
for K in libbih_amd.so variants/libbih_amd_P8.so variants/libbih_amd_P12.so variants/libbih_amd_P24.so; do
  for T in anyhit reference; do
    BIH_LIB=bih-gpu-raytracer_amd/lib/$K timeout -k 10 120 python tools/time_render.py --traverse $T --tag "$K" >> gpurun_out/ab5.jsonl 2>/dev/null || echo "fail $K $T"
  done
done
cat gpurun_out/ab5.jsonl | cut -c1-200
