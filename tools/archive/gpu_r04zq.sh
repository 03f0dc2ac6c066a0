set -u
for T in 1 0 1 0; do
  BIH_TREE_STREAM=$T timeout -k 10 300 python -u bench.py --no-reference-leg --c5 0 --whitted-frames 0 --cpu-baseline 0 --traffic 0 > gpurun_out/bq_r04zq_t$T.json 2>gpurun_out/bq_r04zq_t$T.err || { tail -5 gpurun_out/bq_r04zq_t$T.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'head %.4f' % d['ms_per_step'], 'one %.4f' % d['one_in_flight']['ms_per_step'], 'cam %.4f' % d['moving_camera']['ms_per_step'], 'rb %.4f' % d['with_rebuild']['ms_per_step'])
" gpurun_out/bq_r04zq_t$T.json t$T | tee -a gpurun_out/bq_r04zq.txt
done
