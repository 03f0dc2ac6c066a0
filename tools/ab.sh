# usage: bash tools/ab.sh OUTFILE LIB... ; times tile and refill kernels for each lib variant
set -u
OUT=$1; shift
for K in "$@"; do
  for V in tile refill; do
    BIH_LIB=bih-gpu-raytracer_amd/lib/$K BIH_RENDER_KERNEL=$V timeout -k 10 120 python tools/time_render.py --tag "$K" >> "$OUT" 2>/dev/null || echo "fail $K $V"
  done
done
cat "$OUT"
