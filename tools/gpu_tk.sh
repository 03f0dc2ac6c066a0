# GPU parity tests, then the per-camera kernel profile (tools/gpu_kcam.sh)
# and the bench line; stops at the first failure.  usage: bash tools/gpu_tk.sh TAG
set -u
T=$1
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > $R/gpurun_out/${T}_tests.log 2>&1; rc=$?
tail -3 $R/gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit 1
bash $R/tools/gpu_kcam.sh ${T} > $R/gpurun_out/${T}_kcam.txt 2>&1 || exit 1
cd $R && timeout -k 10 700 python -u bench.py --cpu-baseline 0 > $R/gpurun_out/${T}_bench.json 2> $R/gpurun_out/${T}_bench.err || exit 1
cut -c1-300 $R/gpurun_out/${T}_bench.json
