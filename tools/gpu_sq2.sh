# SQ counters of k_render_bins per launch (tools/prof_render.py), one
# rocprofv3 pass per frames-per-call setting.  usage: bash tools/gpu_sq2.sh TAG
set -u
T=$1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for g in 1 16; do
  timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d $R/gpurun_out/prof_${T}_g$g/sq1 -o sq1 --output-format csv -- python3 $R/tools/prof_render.py --frames 4 --group $g \
    > $R/gpurun_out/prof_${T}_g${g}_sq1.log 2>&1 || exit 1
  echo "== group $g"
  python3 $R/tools/summarize_prof.py $R/gpurun_out/prof_${T}_g$g k_render_bins || exit 1
done
