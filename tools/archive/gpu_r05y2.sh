# Round 5: per-dispatch trace of the bench's roofline samples (isolated
# 16-frame calls rotating over 3 streams: ring instance, shared grid)
set -u
T=${1:-r05y}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/g16_rot -o k --output-format csv -- \
    python3 $R/tools/call_breakdown.py --frames 16 --calls 20 --sync 1 --streams 3 > $O/g16_rot.log 2>&1 || exit 1
python3 $R/tools/call_timeline.py $O/g16_rot/k_kernel_trace.csv --show 1 --dispatch-csv $O/g16_rot_dispatches.csv > $O/g16_rot_timeline.txt
tail -8 $O/g16_rot_timeline.txt
