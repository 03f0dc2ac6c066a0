# Round 5: where a rebuild + render step goes (kernel trace of the bench's
# with_rebuild window)
set -u
T=${1:-r05ab}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/rb -o k --output-format csv -- \
    python3 $R/tools/rb_window.py --repeat 2 > $O/rb.log 2>&1 || { tail -20 $O/rb.log; exit 1; }
python3 $R/tools/window_timeline.py $O/rb/k_kernel_trace.csv $O/rb.log > $O/rb_timeline.txt
python3 $R/tools/window_timeline.py $O/rb/k_kernel_trace.csv $O/rb.log --quiet | tail -24
