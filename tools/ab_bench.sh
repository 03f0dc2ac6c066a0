# usage: bash tools/ab_bench.sh TAG VARIANT...: bench.py headline (frames in
# flight, no side legs) for the default library and each variant, twice in
# alternation; prints ms_per_step per run.
set -u
TAG=$1; shift
J=gpurun_out/abb_$TAG.txt; rm -f $J
for rep in 1 2; do
  for V in default "$@"; do
    if [ "$V" = default ]; then L=""; else L=bih-gpu-raytracer_amd/lib/variants/libbih_amd_$V.so; fi
    BIH_LIB=$L timeout -k 10 200 python bench.py --steps 60 --warmup 5 --traffic 0 --cpu-baseline 0 \
      --no-reference-leg --no-rebuild-leg > gpurun_out/abb_${TAG}_$V.json 2>/dev/null || { echo "fail $V"; exit 1; }
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], round(d['ms_per_step'],4), round(d['kernel_ms'],3), round(d['one_in_flight']['ms_per_step'],4))" gpurun_out/abb_${TAG}_$V.json $V | tee -a $J
  done
done
