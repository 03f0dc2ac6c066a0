# A/B of the default 1080p headline (bench.py --headline-only) between the
# tree's library and variant libraries (tools/build_variants.sh), alternating.
# usage: bash tools/gpu_habn.sh TAG ROUNDS VARIANT...
set -u
TAG=$1; N=$2; shift 2
R=$GRAFT_REPO_ROOT
A="--steps 1000 --warmup 50 --headline-only --traffic 0 --cpu-baseline 0"
for k in $(seq 1 $N); do
  for V in head "$@"; do
    if [ "$V" = head ]; then L=""; else L=$R/bih-gpu-raytracer_amd/lib/variants/libbih_amd_$V.so; fi
    BIH_LIB=$L timeout -k 10 300 python -u bench.py $A > gpurun_out/habn_${TAG}_${V}_$k.json 2>gpurun_out/habn_${TAG}_${V}_$k.err || exit 1
    python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], round(d['value']/1e9,2), d.get('kernel_ms'))
" gpurun_out/habn_${TAG}_${V}_$k.json $V | tee -a gpurun_out/habn_$TAG.txt
  done
done
