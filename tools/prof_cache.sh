# scalar-cache / L2 counters of the render kernel (one counter group per pass)
set -u
TAG=$1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for G in "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQC_DCACHE_MISSES_DUPLICATE" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" "SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU" "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $G -d $R/gpurun_out/prof_$TAG/p$i -o p$i --output-format csv -- python3 $R/tools/prof_render.py --frames 3 > $R/gpurun_out/prof_$TAG/p$i.log 2>&1
  echo "pass $i rc=$?"
done
