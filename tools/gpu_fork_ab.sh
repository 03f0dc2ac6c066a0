# A/B of variant libraries on one-frame calls (ab_group G=1, 1 in flight),
# the pipelined headline and the bench's per-step legs.
# usage: bash tools/gpu_fork_ab.sh TAG VARIANT...
set -u
T=$1; shift
R=$GRAFT_REPO_ROOT
for k in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then L=""; else L="BIH_LIB=$R/bih-gpu-raytracer_amd/lib/variants/libbih_amd_$v.so"; fi
    echo "== g1 $v $(env $L timeout -k 10 120 python3 $R/tools/ab_group.py --frames 600 --group 1 --in-flight 1 2>/dev/null | tail -1)"
    echo "== g16 $v $(env $L timeout -k 10 120 python3 $R/tools/ab_group.py --frames 1600 --group 16 --in-flight 3 2>/dev/null | tail -1)"
    env $L timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --traffic 0 --cpu-baseline 0 --c5 0 --whitted-frames 0 --no-reference-leg --share-world 1 > gpurun_out/${T}_${v}_$k.json 2>/dev/null || exit 1
    python3 -c "
import json
d=json.loads(open('gpurun_out/${T}_${v}_$k.json').read().strip().splitlines()[-1])
print('== legs $v', round(d['ms_per_step'],5), 'serial', round(d['one_in_flight']['ms_per_step'],5), 'moving', round(d['moving_camera']['ms_per_step'],4), 'rebuild', round(d['with_rebuild']['ms_per_step'],4))
"
  done
done
