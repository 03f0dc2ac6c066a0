# A/B of the C5 headline (10M tris, 3840x2160) between a variant library
# (tools/build_rev_variant.sh NAME REV) and the tree's own, alternating.
# usage: bash tools/gpu_c5ab.sh NAME
set -u
V=$1
R=$GRAFT_REPO_ROOT
A="--tris 10000000 --width 3840 --height 2160 --steps 100 --warmup 10 --headline-only --traffic 0 --cpu-baseline 0"
for k in 1 2; do
  BIH_LIB=$R/bih-gpu-raytracer_amd/lib/variants/libbih_amd_$V.so timeout -k 10 300 python -u bench.py $A > gpurun_out/c5ab_${V}_$k.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py $A > gpurun_out/c5ab_head_$k.json 2>/dev/null || exit 1
  python3 -c "
import json
for n in ('${V}_$k','head_$k'):
    d=json.loads(open('gpurun_out/c5ab_'+n+'.json').read().strip().splitlines()[-1]); print(n, d['ms_per_step'], d['value']/1e9)
"
done
