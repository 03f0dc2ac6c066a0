# Round 5: knob sweep -- items per tile in share launches (BIH_ITEM_TILES)
# and blocks per CU of a lone launch (BIH_BINS_BLOCKS_PER_CU).
set -u
T=${1:-r05af}
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_ab5.sh $T 2 base base+BIH_ITEM_TILES=131072 base+BIH_ITEM_TILES=32768 base+BIH_BINS_BLOCKS_PER_CU=5 || exit 1
