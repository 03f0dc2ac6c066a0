set -u
R=$GRAFT_REPO_ROOT
bash tools/gpu_ab5.sh r05i 2 base hf15 hf12 || exit 1
O=$R/gpurun_out/r05i
V=$R/bih-gpu-raytracer_amd/lib/variants
rm -f $O/tl.bin
BIH_LIB=$V/libbih_amd_tl.so BIH_TIMELINE_OUT=$O/tl.bin timeout -k 10 120 python3 tools/call_breakdown.py --frames 16 --calls 4 --warm 4 > $O/tl.log 2>&1 || exit 1
python3 tools/bins_timeline.py $O/tl.bin --skip 4 --show 1 | tee $O/tl_g16.txt | head -40
