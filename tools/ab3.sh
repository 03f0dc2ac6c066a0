set -u
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout=300 -x > gpurun_out/t7.log 2>&1; echo tests_packet_rc=$?; tail -3 gpurun_out/t7.log
for V in packet tile; do
  for K in libbih_amd.so variants/libbih_amd_P8.so variants/libbih_amd_P12.so variants/libbih_amd_K8.so; do
    BIH_LIB=bih-gpu-raytracer_amd/lib/$K BIH_RENDER_KERNEL=$V timeout -k 10 120 python tools/time_render.py --tag "$K" >> gpurun_out/ab4.jsonl 2>/dev/null || echo "fail $K $V"
  done
done
BIH_RENDER_KERNEL=packet timeout -k 10 120 python tools/time_render.py --traverse reference --tag ref >> gpurun_out/ab4.jsonl 2>/dev/null
cat gpurun_out/ab4.jsonl | cut -c1-230
