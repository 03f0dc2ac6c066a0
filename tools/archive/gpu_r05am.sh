# Round 5: renders after a rebuild take 1 / 2 / 3 blocks per CU
# (BIH_BINS_REBUILD_PER_CU; BIH_REBUILD_GRID=0 off) -- A/B and the rebuild
# window.
set -u
T=${1:-r05am}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
bash tools/gpu_ab5.sh $T 2 base base+BIH_REBUILD_GRID=0 base+BIH_BINS_REBUILD_PER_CU=1 base+BIH_BINS_REBUILD_PER_CU=3 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/rb -o k --output-format csv -- \
    python3 $R/tools/rb_window.py --repeat 2 > $O/rb.log 2>&1 || { tail -20 $O/rb.log; exit 1; }
python3 $R/tools/window_timeline.py $O/rb/k_kernel_trace.csv $O/rb.log > $O/rb_timeline.txt
grep "ms_per_step" $O/rb.log
