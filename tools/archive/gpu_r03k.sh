set -u
export TMPDIR=/tmp
T=r03k
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for g in 1 4 8; do
  timeout -k 10 600 python bench.py --steps 400 --warmup 40 --group $g --traffic 0 --cpu-baseline 0 --whitted-frames 0 --no-reference-leg --no-rebuild-leg > gpurun_out/${T}_g$g.json 2> gpurun_out/${T}_g$g.err || { tail -20 gpurun_out/${T}_g$g.err; exit 1; }
  echo "group $g"; python tools/bench_summary.py gpurun_out/${T}_g$g.json | head -4
done
