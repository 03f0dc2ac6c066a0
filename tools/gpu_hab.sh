# A/B of the default 1080p headline between a variant library
# (tools/build_rev_variant.sh NAME REV) and the tree's own, alternating.
# usage: bash tools/gpu_hab.sh NAME [ROUNDS]
set -u
V=$1; N=${2:-3}
R=$GRAFT_REPO_ROOT
A="--steps 1000 --warmup 50 --headline-only --traffic 0 --cpu-baseline 0"
for k in $(seq 1 $N); do
  BIH_LIB=$R/bih-gpu-raytracer_amd/lib/variants/libbih_amd_$V.so timeout -k 10 300 python -u bench.py $A > gpurun_out/hab_${V}_$k.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py $A > gpurun_out/hab_head_$k.json 2>/dev/null || exit 1
  python3 -c "
import json
for n in ('${V}_$k','head_$k'):
    d=json.loads(open('gpurun_out/hab_'+n+'.json').read().strip().splitlines()[-1]); print(n, d['ms_per_step'], d['value']/1e9)
"
done
