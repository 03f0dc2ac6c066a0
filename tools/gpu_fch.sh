# fast counters + per-phase wave cycles of two variants on 16-frame calls
set -u
for V in "$@"; do
  BIH_LIB=bih-gpu-raytracer_amd/lib/variants/libbih_amd_$V.so timeout -k 10 120 python tools/fast_counters.py --frames 3 --group 16 > gpurun_out/fch_$V.log 2>&1 || exit 1
  echo "== $V"; grep -E "bin-phases|bins:" gpurun_out/fch_$V.log | tail -2
done
