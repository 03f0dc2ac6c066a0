# Round 5: queue refill batch 4 (BIH_BIN_BATCH) and 4 render slots
# (BIH_RENDER_SLOTS) against the defaults (8, 3).
set -u
T=${1:-r05al}
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_ab5.sh $T 2 base bb4 sl4 || exit 1
