# usage: bash tools/ab_inflight.sh TAG: frames in flight 2 (default lib) vs 3/4
# (libs built with BIH_RENDER_SLOTS=3/4), bench headline only, twice each.
set -u
TAG=$1
J=gpurun_out/abf_$TAG.txt; rm -f $J
for rep in 1 2; do
  for F in 2 3 4; do
    if [ $F = 2 ]; then L=""; else L=bih-gpu-raytracer_amd/lib/variants/libbih_amd_slots$F.so; fi
    BIH_LIB=$L timeout -k 10 200 python bench.py --steps 60 --warmup 5 --traffic 0 --cpu-baseline 0 \
      --no-reference-leg --no-rebuild-leg --in-flight $F > gpurun_out/abf_${TAG}_$F.json 2>gpurun_out/abf_${TAG}_$F.err || { echo "fail $F"; exit 1; }
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('inflight', sys.argv[2], round(d['ms_per_step'],4), round(d['kernel_ms'],3), round(d['one_in_flight']['ms_per_step'],4))" gpurun_out/abf_${TAG}_$F.json $F | tee -a $J
  done
done
