# Round 5: tests (with the ring jump-table test) and the shared grid's blocks
# per CU under the alternating-stream rule (A/B 3 / 4 / 5).
set -u
T=${1:-r05ac}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --durations=5 --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab5.sh $T 2 base base+BIH_BINS_MULTI_PER_CU=5 base+BIH_BINS_MULTI_PER_CU=3 || exit 1
