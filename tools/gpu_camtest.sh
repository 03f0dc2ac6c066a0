# GPU parity tests + the per-camera kernel profile + SQ counters of it.
# usage: bash tools/gpu_camtest.sh TAG
set -u
T=$1
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
bash tools/gpu_kcam_build.sh ${T} || exit 1
bash tools/gpu_sqcam.sh ${T}
