# Round 5: item timelines with per-item work counters (what makes a tile slow)
set -u
T=${1:-r05g}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
V=$R/bih-gpu-raytracer_amd/lib/variants
tl() {   # tl NAME COST ARGS...
  local N=$1; local C=$2; shift 2
  rm -f $O/$N.bin
  BIH_COST_QUEUE=$C BIH_LIB=$V/libbih_amd_tl.so BIH_TIMELINE_OUT=$O/$N.bin timeout -k 10 120 python3 tools/call_breakdown.py "$@" > $O/$N.log 2>&1 || { tail -20 $O/$N.log; return 1; }
  grep "^calls" $O/$N.log
  python3 tools/bins_timeline.py $O/$N.bin --skip 4 --show 1 > $O/${N}_tl.txt; cat $O/${N}_tl.txt
}
tl tl_g16_cost 1 --frames 16 --calls 4 --warm 4 &&
tl tl_one_cost 1 --frames 1 --calls 8 --warm 4
