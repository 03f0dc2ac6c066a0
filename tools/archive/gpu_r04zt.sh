set -u
for B in 0 5 0 5; do
  if [ $B = 0 ]; then unset BIH_BINS_BLOCKS_PER_CU; else export BIH_BINS_BLOCKS_PER_CU=$B; fi
  timeout -k 10 300 python -u bench.py --no-reference-leg --c5 0 --whitted-frames 0 --cpu-baseline 0 --traffic 0 > gpurun_out/bq_r04zt_b$B.json 2>/dev/null || exit 1
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'head %.4f' % d['ms_per_step'], 'launch %.4f' % (d['roofline']['launch_ms']/16), 'one %.4f' % d['one_in_flight']['ms_per_step'], 'cam %.4f' % d['moving_camera']['ms_per_step'], 'rb %.4f' % d['with_rebuild']['ms_per_step'])
" gpurun_out/bq_r04zt_b$B.json b$B | tee -a gpurun_out/bq_r04zt.txt
done
