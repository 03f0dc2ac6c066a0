# Round-4 check: bash tools/gpu_r04d.sh TAG VARIANT...
# all gpu tests, the driver's bench command, rocprof of the headline, the
# headline A/B (G=16, 3 in flight) and the one-frame A/B (G=1, 1 in flight)
# against variant libraries, build/camera kernel profiles, C4 with and without
# the bounce-queue ray order.
set -u
T=$1; shift
R=$GRAFT_REPO_ROOT
bash tools/gpu_r04.sh $T "" --gpus 1 --steps 20 --warmup 5 || exit 1
bash tools/gpu_hab2.sh ${T}_ab 2 "$@" || exit 1
for v in default "$@"; do
  if [ $v = default ]; then L=""; else L="BIH_LIB=$R/bih-gpu-raytracer_amd/lib/variants/libbih_amd_$v.so"; fi
  echo "== g1 $v $(env $L timeout -k 10 120 python3 $R/tools/ab_group.py --frames 400 --group 1 --in-flight 1 2>/dev/null | tail -1)"
done
bash tools/gpu_kcam_build.sh ${T}_k || exit 1
cd $R
for s in 1 0; do
  BIH_WH_SORT=$s timeout -k 10 300 python3 $R/tools/time_whitted.py --frames 2 > $R/gpurun_out/${T}_wh_sort$s.json 2>/dev/null || exit 1
  echo "== wh sort=$s $(tail -1 $R/gpurun_out/${T}_wh_sort$s.json | cut -c1-300)"
done
