set -u
R=$GRAFT_REPO_ROOT
bash tools/gpu_ab5.sh r05j 2 base prev2 hf0 || exit 1
O=$R/gpurun_out/r05j
V=$R/bih-gpu-raytracer_amd/lib/variants
for F in 16 1; do
rm -f $O/tl$F.bin
BIH_LIB=$V/libbih_amd_tl.so BIH_TIMELINE_OUT=$O/tl$F.bin timeout -k 10 120 python3 tools/call_breakdown.py --frames $F --calls 4 --warm 4 > $O/tl$F.log 2>&1 || exit 1
python3 tools/bins_timeline.py $O/tl$F.bin --skip 4 --show 1 | tee $O/tl_g$F.txt | head -12
done
