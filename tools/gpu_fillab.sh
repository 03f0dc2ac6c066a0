# GPU tests, per-camera kernel times, headline A/B against lib variants.
# usage: bash tools/gpu_fillab.sh TAG ROUNDS VARIANT...
set -u
T=$1; N=$2; shift 2
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
bash tools/gpu_varcam.sh ${T} base "$@" || exit 1
cd $R && bash tools/gpu_ab.sh ${T} $N "$@"
