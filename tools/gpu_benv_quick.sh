# bench.py (headline + one-frame, moving-camera and rebuild legs; no reference,
# C4, C5 or CPU legs) for the tree's library and variants, alternating.
# usage: bash tools/gpu_benv_quick.sh TAG ROUNDS VARIANT...
set -u
TAG=$1; N=$2; shift 2
R=$GRAFT_REPO_ROOT
for k in $(seq 1 $N); do
  for V in head "$@"; do
    if [ "$V" = head ]; then L=""; else L=$R/bih-gpu-raytracer_amd/lib/variants/libbih_amd_$V.so; fi
    BIH_LIB=$L timeout -k 10 300 python -u bench.py --no-reference-leg --c5 0 --whitted-frames 0 --cpu-baseline 0 --traffic 0 \
      > gpurun_out/bq_${TAG}_${V}_$k.json 2>gpurun_out/bq_${TAG}_${V}_$k.err || exit 1
    python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'head %.4f' % d['ms_per_step'], 'one %.4f' % d['one_in_flight']['ms_per_step'], 'cam %.4f' % d['moving_camera']['ms_per_step'], 'rb %.4f' % d['with_rebuild']['ms_per_step'], 'share %.5f' % max(d['band_share']['share_ms_per_step']))
" gpurun_out/bq_${TAG}_${V}_$k.json $V | tee -a gpurun_out/bq_$TAG.txt
  done
done
