# usage: bash tools/ab_bench_env.sh TAG "ENV=.." ["ENV=.." ...]: bench.py headline
# (frames in flight, no side legs) per environment setting, twice in
# alternation; prints ms_per_step, kernel_ms and the one-in-flight ms.
# "-" runs the default environment.
set -u
TAG=$1; shift
J=gpurun_out/abe_$TAG.txt; rm -f $J
i=0
for rep in 1 2; do
  for E in "$@"; do
    i=$((i+1))
    [ "$E" = "-" ] && E="BIH_AB_DEFAULT=1"
    env $E timeout -k 10 200 python bench.py --steps 60 --warmup 5 --traffic 0 --cpu-baseline 0 \
      --no-reference-leg --no-rebuild-leg > gpurun_out/abe_${TAG}_$i.json 2>gpurun_out/abe_${TAG}_$i.err || { echo "fail $E"; exit 1; }
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], round(d['ms_per_step'],4), round(d['kernel_ms'],3), round(d['one_in_flight']['ms_per_step'],4))" gpurun_out/abe_${TAG}_$i.json "$E" | tee -a $J
  done
done
