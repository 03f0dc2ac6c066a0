# Round 5: fused advance on/off vs prev (driver command), item timelines
# (per-wave records), C4 with/without the bins mask.
set -u
T=${1:-r05d}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
V=$R/bih-gpu-raytracer_amd/lib/variants
for k in 1 2; do
  for X in fused nofused prev; do
    L=""; E=""
    [ $X = prev ] && L=$V/libbih_amd_prev.so
    [ $X = nofused ] && E=0
    BIH_LIB=$L BIH_FUSED_ADVANCE=${E:-1} timeout -k 10 300 python -u bench.py --c5 0 --whitted-frames 0 \
        --cpu-baseline 0 --traffic 0 --no-reference-leg > $O/bench_${X}_$k.json 2> $O/bench_${X}_$k.err || { tail -20 $O/bench_${X}_$k.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'head %.4f' % d['ms_per_step'], 'launch %.4f' % (d['roofline']['launch_ms']/16), 'one %.4f' % d['one_in_flight']['ms_per_step'], 'cam %.4f' % d['moving_camera']['ms_per_step'], 'rb %.4f' % d['with_rebuild']['ms_per_step'], 'share %.3f' % d['band_share']['projected_efficiency'], 'c2 %.4f' % d['c2_torus']['ms_per_step'])
" $O/bench_${X}_$k.json $X | tee -a $O/ab.txt
  done
done
for X in mask nomask prev; do
  L=""; E=1
  [ $X = prev ] && L=$V/libbih_amd_prev.so
  [ $X = nomask ] && E=0
  BIH_LIB=$L BIH_WH_BINS=$E timeout -k 10 200 python3 tools/time_whitted.py --frames 3 > $O/wh_$X.log 2>&1 || { tail -20 $O/wh_$X.log; exit 1; }
  echo "$X $(tail -1 $O/wh_$X.log)" | tee -a $O/ab.txt
done
tl() {   # tl NAME FUSED ARGS...
  local N=$1; local F=$2; shift 2
  rm -f $O/$N.bin
  BIH_FUSED_ADVANCE=$F BIH_LIB=$V/libbih_amd_tl.so BIH_TIMELINE_OUT=$O/$N.bin timeout -k 10 120 python3 tools/call_breakdown.py "$@" > $O/$N.log 2>&1 || { tail -20 $O/$N.log; return 1; }
  grep "^calls" $O/$N.log
  python3 tools/bins_timeline.py $O/$N.bin --skip 4 --show 1 > $O/${N}_tl.txt; tail -25 $O/${N}_tl.txt
}
tl tl_one_nf 0 --frames 1 --calls 16 --warm 4 &&
tl tl_g16_nf 0 --frames 16 --calls 6 --warm 4 &&
tl tl_g16_f 1 --frames 16 --calls 6 --warm 4 &&
tl tl_share8_g16_nf 0 --frames 16 --calls 6 --warm 4 --share 0/8
