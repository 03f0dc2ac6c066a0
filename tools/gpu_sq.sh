# SQ / TCC counters of the default render (tools/prof_render.py), one pass per group
set -u
T=$1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d $R/gpurun_out/prof_${T}/sq1 -o sq1 --output-format csv -- python3 $R/tools/prof_render.py --frames 3 > $R/gpurun_out/prof_${T}_sq1.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_SCA \
  -d $R/gpurun_out/prof_${T}/sq2 -o sq2 --output-format csv -- python3 $R/tools/prof_render.py --frames 3 > $R/gpurun_out/prof_${T}_sq2.log 2>&1 || \
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_INSTS_LDS \
  -d $R/gpurun_out/prof_${T}/sq2 -o sq2 --output-format csv -- python3 $R/tools/prof_render.py --frames 3 > $R/gpurun_out/prof_${T}_sq2.log 2>&1 || exit 1
python3 $R/tools/summarize_prof.py $R/gpurun_out/prof_${T} k_render_bins || true
