set -u
for cfg in "4 0" "3 0" "2 0" "4 5" "4 4"; do
  set -- $cfg; M=$1; S=$2
  export BIH_BINS_MULTI_PER_CU=$M
  if [ $S = 0 ]; then unset BIH_BINS_BLOCKS_PER_CU; else export BIH_BINS_BLOCKS_PER_CU=$S; fi
  timeout -k 10 300 python -u bench.py --no-reference-leg --c5 0 --whitted-frames 0 --cpu-baseline 0 --traffic 0 > gpurun_out/bq_r04zl_m${M}s$S.json 2>gpurun_out/bq_r04zl_m${M}s$S.err || exit 1
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'head %.4f' % d['ms_per_step'], 'launch %.4f' % (d['roofline']['launch_ms']/16), 'one %.4f' % d['one_in_flight']['ms_per_step'], 'cam %.4f' % d['moving_camera']['ms_per_step'], 'rb %.4f' % d['with_rebuild']['ms_per_step'], 'share %.5f' % max(d['band_share']['share_ms_per_step']))
" gpurun_out/bq_r04zl_m${M}s$S.json m${M}s$S | tee -a gpurun_out/bq_r04zl.txt
done
