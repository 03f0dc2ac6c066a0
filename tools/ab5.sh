set -u
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout=300 -x > gpurun_out/t9.log 2>&1; echo tests_rc=$?; tail -3 gpurun_out/t9.log
for K in libbih_amd.so variants/libbih_amd_P8.so variants/libbih_amd_P4.so; do
  for T in anyhit reference; do
    BIH_LIB=bih-gpu-raytracer_amd/lib/$K timeout -k 10 120 python tools/time_render.py --traverse $T --tag "$K" >> gpurun_out/ab6.jsonl 2>/dev/null || echo "fail $K $T"
  done
done
cat gpurun_out/ab6.jsonl | cut -c1-200
