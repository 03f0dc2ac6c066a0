# Round 5: SGPR cap on k_render_bins (room for the next call's advance beside
# the render; the stamped instance at 6 waves) -- A/B, window traces.
set -u
T=${1:-r05v}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
V=$R/bih-gpu-raytracer_amd/lib/variants
bash tools/gpu_ab5.sh $T 2 base sg96 sg80 || exit 1
cd /tmp && export TMPDIR=/tmp
win() {   # win NAME LIB ARGS...
  local N=$1; local L=$2; shift 2
  BIH_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace -d $O/$N -o k --output-format csv -- \
      python3 $R/tools/window_trace.py "$@" > $O/$N.log 2>&1 || { tail -20 $O/$N.log; return 1; }
  python3 $R/tools/window_timeline.py $O/$N/k_kernel_trace.csv $O/$N.log > $O/${N}_timeline.txt
  tail -9 $O/${N}_timeline.txt
}
win full_sg96 $V/libbih_amd_sg96.so --repeat 3 &&
win share0_sg96 $V/libbih_amd_sg96.so --share 0/8 --repeat 3
