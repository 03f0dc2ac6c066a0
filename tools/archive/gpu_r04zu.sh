set -u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "render or frames or camera or rebuild" > gpurun_out/r04zu_tests.log 2>&1 || { tail -40 gpurun_out/r04zu_tests.log; exit 1; }
tail -1 gpurun_out/r04zu_tests.log
for k in 1 2; do
  for V in head prev; do
    if [ "$V" = head ]; then L=""; else L=$GRAFT_REPO_ROOT/bih-gpu-raytracer_amd/lib/variants/libbih_amd_$V.so; fi
    BIH_LIB=$L timeout -k 10 300 python -u bench.py --no-reference-leg --c5 0 --whitted-frames 0 --cpu-baseline 0 --traffic 0 > gpurun_out/bq_r04zu_${V}_$k.json 2>/dev/null || exit 1
    python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'head %.4f' % d['ms_per_step'], 'launch %.4f' % (d['roofline']['launch_ms']/16), 'one %.4f' % d['one_in_flight']['ms_per_step'], 'cam %.4f' % d['moving_camera']['ms_per_step'], 'rb %.4f' % d['with_rebuild']['ms_per_step'])
" gpurun_out/bq_r04zu_${V}_$k.json $V | tee -a gpurun_out/bq_r04zu.txt
  done
done
