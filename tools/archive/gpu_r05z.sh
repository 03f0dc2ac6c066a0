# Round 5: shared grid when the caller alternates streams -- A/B, windows.
set -u
T=${1:-r05z}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
bash tools/gpu_ab5.sh $T 2 base base+BIH_SHARE_ALTERNATING=0 || exit 1
cd /tmp && export TMPDIR=/tmp
win() {   # win NAME TOOL ARGS...
  local N=$1; local P=$2; shift 2
  timeout -k 10 180 rocprofv3 --kernel-trace -d $O/$N -o k --output-format csv -- \
      python3 $R/tools/$P "$@" > $O/$N.log 2>&1 || { tail -20 $O/$N.log; return 1; }
  python3 $R/tools/window_timeline.py $O/$N/k_kernel_trace.csv $O/$N.log > $O/${N}_timeline.txt
}
win full window_trace.py --repeat 3 && tail -9 $O/full_timeline.txt | head -9 &&
win share0 window_trace.py --share 0/8 --repeat 3 && grep -A9 "^window 2" $O/share0_timeline.txt | head -9
