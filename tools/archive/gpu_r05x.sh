# Round 5: tile costs measured from a camera's second render on -- tests,
# A/B against HEAD, moving-camera window.
set -u
T=${1:-r05x}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --durations=5 --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab5.sh $T 2 base hd || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/cam -o k --output-format csv -- \
    python3 $R/tools/cam_window.py --repeat 2 > $O/cam.log 2>&1 || { tail -20 $O/cam.log; exit 1; }
python3 $R/tools/window_timeline.py $O/cam/k_kernel_trace.csv $O/cam.log > $O/cam_timeline.txt
python3 $R/tools/window_timeline.py $O/cam/k_kernel_trace.csv $O/cam.log --quiet | tail -19
