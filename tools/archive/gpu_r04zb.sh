set -u
for G in 1 16; do
  BIH_LIB=bih-gpu-raytracer_amd/lib/variants/libbih_amd_fc.so timeout -k 10 120 python tools/fast_counters.py --frames 3 --group $G > gpurun_out/r04zb_fc_g$G.log 2>&1 || exit 1
  echo "== group $G"; grep -E "bin-phases|bin-counters" gpurun_out/r04zb_fc_g$G.log | tail -2
done
bash tools/gpu_sqcam.sh r04zb
