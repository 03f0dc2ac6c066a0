set -u
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout=300 -x > gpurun_out/t10.log 2>&1; echo tests_rc=$?; tail -3 gpurun_out/t10.log
rm -f gpurun_out/ab7.jsonl
for K in packet packet1; do
  for T in anyhit reference; do
    BIH_RENDER_KERNEL=$K timeout -k 10 120 python tools/time_render.py --traverse $T --tag "$K" >> gpurun_out/ab7.jsonl 2>gpurun_out/ab7.err || echo "fail $K $T"
  done
done
for V in P8 P24; do
  BIH_LIB=bih-gpu-raytracer_amd/lib/variants/libbih_amd_$V.so timeout -k 10 120 python tools/time_render.py --traverse anyhit --tag "$V" >> gpurun_out/ab7.jsonl 2>>gpurun_out/ab7.err || echo "fail $V"
done
cut -c1-220 gpurun_out/ab7.jsonl
