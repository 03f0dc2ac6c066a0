# Round 5: k_render_fallback's grid 64 / 16 / 4 blocks (BIH_FB_BLOCKS)
set -u
T=${1:-r05an}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
bash tools/gpu_ab5.sh $T 2 base fb16 fb4 || exit 1
cd /tmp && export TMPDIR=/tmp
for X in base fb4; do
  L=""; [ $X != base ] && L=$R/bih-gpu-raytracer_amd/lib/variants/libbih_amd_$X.so
  BIH_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/one_$X -o k --output-format csv -- \
      python3 $R/tools/call_breakdown.py --frames 1 --calls 40 --sync 1 > $O/one_$X.log 2>&1 || exit 1
  grep -h "k_render_fallback" $O/one_$X/k_kernel_stats.csv | cut -d, -f2-4 | sed "s/^/$X /"
done
