# Round 5: an item's first list chunk requested beside its state load
# (BIH_ITEM_PREFETCH) -- tests, A/B against the build without it.
set -u
T=${1:-r05aj}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab5.sh $T 3 base pf0 || exit 1
