# SQ counters of the per-camera kernels (tools/prof_camera.py: camera moving
# every frame), one rocprofv3 pass per counter group.
# usage: bash tools/gpu_sqcam.sh TAG
set -u
T=$1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d $R/gpurun_out/sqcam_${T}/p1 -o p1 --output-format csv -- python3 $R/tools/prof_camera.py --frames 8 > $R/gpurun_out/sqcam_${T}_p1.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU \
  -d $R/gpurun_out/sqcam_${T}/p2 -o p2 --output-format csv -- python3 $R/tools/prof_camera.py --frames 8 > $R/gpurun_out/sqcam_${T}_p2.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE \
  -d $R/gpurun_out/sqcam_${T}/p3 -o p3 --output-format csv -- python3 $R/tools/prof_camera.py --frames 8 > $R/gpurun_out/sqcam_${T}_p3.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE \
  -d $R/gpurun_out/sqcam_${T}/p4 -o p4 --output-format csv -- python3 $R/tools/prof_camera.py --frames 8 > $R/gpurun_out/sqcam_${T}_p4.log 2>&1 || exit 1
for k in k_bin_fp k_bin_fill k_bin_count k_tri_prim k_render_bins; do
  echo "== $k"; python3 $R/tools/summarize_prof.py $R/gpurun_out/sqcam_${T} $k | grep -v "calls" || true
done
