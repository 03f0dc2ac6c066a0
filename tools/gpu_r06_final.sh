#!/bin/bash
# Round 6 measurement set: the new stream test, the driver's bench command,
# and rocprofv3 kernel stats of the headline alone (profiles/r06/).
# usage: tools/gpu_r06_final.sh TAG
set -u
T=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "recycled or headline_call_shape" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o head --output-format csv -- \
  python3 $R/bench.py --headline-only --traffic 0 --cpu-baseline 0 --kernel-samples 20 > $O/prof_bench.json 2> $O/prof.err \
  || { tail -30 $O/prof.err; exit 1; }
echo done
