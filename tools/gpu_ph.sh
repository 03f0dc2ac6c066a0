# A/B of variants (tools/gpu_abv.sh) + per-phase wave cycles of the ph variant
# usage: bash tools/gpu_ph.sh TAG [VARIANTS...]
set -u
T=$1; shift
bash tools/gpu_abv.sh $T "$@" || exit 1
PH=bih-gpu-raytracer_amd/lib/variants/libbih_amd_ph.so
BIH_LIB=$PH timeout -k 10 120 python tools/fast_counters.py --frames 2 > gpurun_out/${T}_ph.log 2>&1 || exit 1
grep bin-phases gpurun_out/${T}_ph.log | tail -1
