# Round-4 check + A/Bs: bash tools/gpu_r04c.sh TAG ROUNDS VARIANT...
# gpu_r04.sh (all gpu tests, the driver's bench command, rocprof of the
# headline), the headline A/B against variant libraries, the C4 frame with
# and without the bounce-queue ray order (BIH_WH_SORT).
set -u
T=$1; N=$2; shift 2
R=$GRAFT_REPO_ROOT
bash tools/gpu_r04.sh $T "" --gpus 1 --steps 20 --warmup 5 || exit 1
bash tools/gpu_hab2.sh ${T}_ab $N "$@" || exit 1
bash tools/gpu_kcam_build.sh ${T}_k || exit 1
cd $R
for s in 1 0; do
  BIH_WH_SORT=$s timeout -k 10 300 python3 $R/tools/time_whitted.py --frames 2 > $R/gpurun_out/${T}_wh_sort$s.json 2>/dev/null || exit 1
  echo "== wh sort=$s $(tail -1 $R/gpurun_out/${T}_wh_sort$s.json | cut -c1-300)"
done
for v in default fitpipe0; do
  if [ $v = default ]; then L=""; else L="BIH_LIB=$R/bih-gpu-raytracer_amd/lib/variants/libbih_amd_$v.so"; fi
  echo "== build $v $(env $L timeout -k 10 120 python3 $R/tools/prof_build.py --builds 20 2>/dev/null | tail -1)"
done
