# Round 5: where a moving-camera step goes (kernel trace of the bench's
# moving_camera window, per-kernel sums)
set -u
T=${1:-r05w}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/cam -o k --output-format csv -- \
    python3 $R/tools/cam_window.py --repeat 2 > $O/cam.log 2>&1 || { tail -20 $O/cam.log; exit 1; }
python3 $R/tools/window_timeline.py $O/cam/k_kernel_trace.csv $O/cam.log > $O/cam_timeline.txt
python3 $R/tools/window_timeline.py $O/cam/k_kernel_trace.csv $O/cam.log --quiet | tail -32
