# Round 5: event waits on the stream that recorded the event skipped -- A/B
# against HEAD and the share window.
set -u
T=${1:-r05ag}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
bash tools/gpu_ab5.sh $T 3 base hd || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/share0 -o k --output-format csv -- \
    python3 $R/tools/window_trace.py --share 0/8 --repeat 3 > $O/share0.log 2>&1 || exit 1
python3 $R/tools/window_timeline.py $O/share0/k_kernel_trace.csv $O/share0.log > $O/share0_timeline.txt
grep -A10 "^window 2" $O/share0_timeline.txt | head -10
