# Round-3 GPU check: gpu tests, a full bench (all legs), a kernel-trace profile.
# usage: bash tools/gpu_r03.sh TAG [bench args...]
set -u
T=$1; shift
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 900 python bench.py "$@" > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/${T}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- \
  python bench.py --headline-only --in-flight 1 --steps 96 --warmup 16 --traffic 0 --cpu-baseline 0 \
  > gpurun_out/${T}_prof.log 2>&1 || { tail -20 gpurun_out/${T}_prof.log; exit 1; }
find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/${T}_kernel_stats.csv
head -12 gpurun_out/${T}_kernel_stats.csv | cut -c1-160
