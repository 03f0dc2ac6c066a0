# Kernel trace of a rank's share (8-way split) and of the full frame, 16-frame calls.
# usage: bash tools/gpu_share_prof.sh TAG
set -u
T=$1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for w in 8 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_w$w -o k --output-format csv -- \
      python3 $R/tools/prof_share.py --world $w > $R/gpurun_out/${T}_w$w.log 2>&1 || exit 1
  tail -1 $R/gpurun_out/${T}_w$w.log
done
python3 $R/tools/share_timeline.py $R/gpurun_out/${T}_w8/k_kernel_trace.csv $R/gpurun_out/${T}_w1/k_kernel_trace.csv
