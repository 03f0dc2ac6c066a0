# C4 frame time (tools/time_whitted.py) for the tree's library and variants.
# usage: bash tools/gpu_wh_ab.sh TAG [VARIANT...]
set -u
T=$1; shift
R=$GRAFT_REPO_ROOT
for v in default "$@"; do
  if [ $v = default ]; then L=""; else L="BIH_LIB=$R/bih-gpu-raytracer_amd/lib/variants/libbih_amd_$v.so"; fi
  env $L timeout -k 10 300 python3 $R/tools/time_whitted.py --frames 2 > $R/gpurun_out/${T}_$v.json 2>/dev/null || exit 1
  echo "== $v $(cat $R/gpurun_out/${T}_$v.json | tail -1 | cut -c1-200)"
done
