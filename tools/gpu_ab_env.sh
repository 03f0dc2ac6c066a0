# time_render of the default library under env settings: bash tools/gpu_ab_env.sh TAG "ENV1" "ENV2" ...
set -u
T=$1; shift
J=gpurun_out/${T}_time.jsonl; rm -f $J
for E in "" "$@"; do
  env $E timeout -k 10 120 python tools/time_render.py --tag "[$E]" >> $J 2>/dev/null || { echo "fail $E"; exit 1; }
done
grep -o '"tag[^,]*\|"ms_mean[^,]*' $J
