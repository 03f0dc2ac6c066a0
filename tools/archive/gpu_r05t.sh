# Round 5: the bench's timed window traced (full frame and rank 0 of 8's
# share), host issue times against the kernels.
set -u
T=${1:-r05t}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
win() {   # win NAME ARGS...
  local N=$1; shift
  timeout -k 10 180 rocprofv3 --kernel-trace -d $O/$N -o k --output-format csv -- \
      python3 $R/tools/window_trace.py "$@" > $O/$N.log 2>&1 || { tail -20 $O/$N.log; return 1; }
  python3 $R/tools/window_timeline.py $O/$N/k_kernel_trace.csv $O/$N.log > $O/${N}_timeline.txt
  tail -16 $O/${N}_timeline.txt
}
win full --repeat 3 &&
win share0 --share 0/8 --repeat 3
