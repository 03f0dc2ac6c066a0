# usage: bash tools/ab_env.sh TAG "ENV=.. ENV2=.." ["ENV=.."...]: anyhit timings per env setting
set -u
TAG=$1; shift
J=gpurun_out/abenv_$TAG.jsonl; rm -f $J
for E in "$@"; do
  env $E timeout -k 10 120 python tools/time_render.py --traverse anyhit --frames 20 --tag "$E" >> $J 2>>gpurun_out/abenv_$TAG.err || { echo "fail $E"; exit 1; }
done
cut -c1-160 $J
