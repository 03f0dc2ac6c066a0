# GPU tests, then bench legs per environment setting (camera sets, frames
# per item).  usage: bash tools/gpu_cam_ab.sh TAG "ENV=.. ENV2=.." ...
set -u
export TMPDIR=/tmp
T=$1; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread --durations=6 \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 300 python bench.py --steps 400 --warmup 40 --traffic 0 --cpu-baseline 0 \
    --whitted-frames 0 --no-reference-leg > gpurun_out/${T}_$i.json 2> gpurun_out/${T}_$i.err \
    || { tail -20 gpurun_out/${T}_$i.err; exit 1; }
  echo "== $envs"; python tools/bench_summary.py gpurun_out/${T}_$i.json | grep -E "^value|band_share|moving|rebuild"
done
