# Headline A/B of variant libraries against the tree's own (bench.py
# --headline-only, alternating).  usage: bash tools/gpu_hab2.sh TAG ROUNDS VARIANT...
set -u
T=$1; N=$2; shift 2
R=$GRAFT_REPO_ROOT
A="--steps 1024 --warmup 64 --headline-only --traffic 0 --cpu-baseline 0"
for k in $(seq 1 $N); do
  for v in default "$@"; do
    if [ $v = default ]; then L=""; else L="BIH_LIB=$R/bih-gpu-raytracer_amd/lib/variants/libbih_amd_$v.so"; fi
    env $L timeout -k 10 300 python -u bench.py $A > gpurun_out/${T}_${v}_$k.json 2>/dev/null || exit 1
    python3 -c "
import json
d=json.loads(open('gpurun_out/${T}_${v}_$k.json').read().strip().splitlines()[-1]); print('$v', $k, round(d['ms_per_step'], 5), round(d['value']/1e9, 1))
"
  done
done
