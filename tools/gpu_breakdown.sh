# Where the bins kernel's time goes: bin counters (BIH_FAST_COUNTERS variant),
# render timing of the default library and the NO_VERIFY / SKIP_TRACE
# variants, and SQ counters of the default kernel.  usage: bash tools/gpu_breakdown.sh TAG
set -u
T=$1
R=$GRAFT_REPO_ROOT
V=bih-gpu-raytracer_amd/lib/variants
BIH_LIB=$V/libbih_amd_fc.so timeout -k 10 120 python tools/fast_counters.py --frames 2 > gpurun_out/${T}_fc.log 2>&1 || exit 1
grep counters gpurun_out/${T}_fc.log | tail -2
J=gpurun_out/${T}_time.jsonl; rm -f $J
timeout -k 10 120 python tools/time_render.py --tag default >> $J 2>/dev/null || exit 1
for X in noverify skiptrace; do
  BIH_LIB=$V/libbih_amd_$X.so timeout -k 10 120 python tools/time_render.py --tag $X >> $J 2>/dev/null || exit 1
done
BIH_BINS=0 timeout -k 10 120 python tools/time_render.py --tag nobins >> $J 2>/dev/null || exit 1
grep -o '"tag[^,]*\|"ms_mean[^,]*' $J
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d $R/gpurun_out/prof_${T}/sq1 -o sq1 --output-format csv -- python3 $R/tools/prof_render.py --frames 3 > $R/gpurun_out/prof_${T}_sq1.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_INSTS_LDS SQ_INSTS_FLAT \
  -d $R/gpurun_out/prof_${T}/sq2 -o sq2 --output-format csv -- python3 $R/tools/prof_render.py --frames 3 > $R/gpurun_out/prof_${T}_sq2.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum \
  -d $R/gpurun_out/prof_${T}/tcc -o tcc --output-format csv -- python3 $R/tools/prof_render.py --frames 3 > $R/gpurun_out/prof_${T}_tcc.log 2>&1 || exit 1
python3 $R/tools/summarize_prof.py $R/gpurun_out/prof_${T} k_render_packet_asm || true
