# Frames per k_render_bins item (BIH_ITEM_TILES): GPU tests, then the
# band-share leg (projected strong-scaling efficiency) per setting.
# usage: bash tools/gpu_split.sh TAG [item_tiles...]
set -u
export TMPDIR=/tmp
T=$1; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread --durations=12 \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for it in "$@"; do
  BIH_ITEM_TILES=$it timeout -k 10 300 python bench.py --steps 400 --warmup 40 --traffic 0 --cpu-baseline 0 \
    --whitted-frames 0 --no-reference-leg > gpurun_out/${T}_it$it.json 2> gpurun_out/${T}_it$it.err \
    || { tail -20 gpurun_out/${T}_it$it.err; exit 1; }
  echo "item_tiles $it"; python tools/bench_summary.py gpurun_out/${T}_it$it.json | grep -E "^value|band_share|moving|rebuild"
done
