set -u
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout=300 > gpurun_out/t5.log 2>&1; echo tests_refill_rc=$?; tail -3 gpurun_out/t5.log
BIH_RENDER_KERNEL=tile timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q --timeout=300 -k "render or counters or bands or 1m" > gpurun_out/t5b.log 2>&1; echo tests_tile_rc=$?; tail -3 gpurun_out/t5b.log
for K in variants/libbih_amd_K8.so libbih_amd.so variants/libbih_amd_K12.so variants/libbih_amd_K16.so; do
  for V in tile refill; do
    BIH_LIB=bih-gpu-raytracer_amd/lib/$K BIH_RENDER_KERNEL=$V timeout -k 10 120 python tools/time_render.py --tag ab >> gpurun_out/ab1.jsonl 2>/dev/null || echo "fail $K $V"
  done
done
BIH_RENDER_KERNEL=refill timeout -k 10 120 python tools/time_render.py --traverse reference --tag ref >> gpurun_out/ab1.jsonl 2>/dev/null
BIH_RENDER_KERNEL=tile timeout -k 10 120 python tools/time_render.py --traverse reference --tag ref >> gpurun_out/ab1.jsonl 2>/dev/null
cat gpurun_out/ab1.jsonl
