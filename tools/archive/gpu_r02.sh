# round-2 GPU call: parity tests, the default bench line, rocprofv3 stats of
# the headline leg (isolated launches), one step after another; stops at the
# first failure.  usage: bash tools/gpu_r02.sh TAG
set -u
T=$1
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > $R/gpurun_out/${T}_tests.log 2>&1; rc=$?
tail -4 $R/gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 700 python -u bench.py > $R/gpurun_out/${T}_bench.json 2> $R/gpurun_out/${T}_bench.err || exit 1
cut -c1-600 $R/gpurun_out/${T}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T} -o k --output-format csv -- \
    python3 $R/bench.py --headline-only --in-flight 1 --traffic 0 --cpu-baseline 0 \
    > $R/gpurun_out/prof_${T}.log 2>&1 || exit 1
f=$(find $R/gpurun_out/prof_${T} -name '*kernel_stats.csv' | head -1)
cut -d, -f1-8 "$f" | head -12
tail -1 $R/gpurun_out/prof_${T}.log | cut -c1-300
