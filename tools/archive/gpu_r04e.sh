# Round-4 check: bash tools/gpu_r04e.sh TAG
# all gpu tests, the driver's bench command, rocprof of the headline,
# build/camera kernel profiles, C4 with and without the bounce-queue ray
# order, SQ counters of k_render_bins.
set -u
T=$1; shift
R=$GRAFT_REPO_ROOT
bash tools/gpu_r04.sh $T "" --gpus 1 --steps 20 --warmup 5 || exit 1
bash tools/gpu_kcam_build.sh ${T}_k || exit 1
cd $R
for s in 1 0; do
  BIH_WH_SORT=$s timeout -k 10 300 python3 $R/tools/time_whitted.py --frames 2 > $R/gpurun_out/${T}_wh_sort$s.json 2>/dev/null || exit 1
  echo "== wh sort=$s $(tail -1 $R/gpurun_out/${T}_wh_sort$s.json | cut -c1-300)"
done
bash tools/gpu_sq2.sh $T || exit 1
