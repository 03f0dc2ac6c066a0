# Round 5: new/changed GPU tests, k_render_bins item timelines, device-count probe.
set -u
T=${1:-r05b}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 300 --timeout-method thread \
    -k "reserved_share or failed_back_tree or headline_call_shape or 10m_4k or whitted_4k or steady_frame" \
    > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed|s call" $O/pytest.log | tail -20
python3 -c "import sys; sys.path.insert(0,'.'); import bench; print('visible_gpu_count', bench.visible_gpu_count())"
python3 -c "import torch; print('torch device_count', torch.cuda.device_count())"
ls /sys/class/kfd/kfd/topology/nodes/ 2>&1 | head; grep -h simd_count /sys/class/kfd/kfd/topology/nodes/*/properties 2>&1 | head -20
echo "ROCR=${ROCR_VISIBLE_DEVICES-unset} HIP=${HIP_VISIBLE_DEVICES-unset} CUDA=${CUDA_VISIBLE_DEVICES-unset}"
L=$R/bih-gpu-raytracer_amd/lib/variants/libbih_amd_tl.so
tl() {   # tl NAME ARGS...
  local N=$1; shift
  rm -f $O/$N.bin
  BIH_LIB=$L BIH_TIMELINE_OUT=$O/$N.bin timeout -k 10 120 python3 tools/call_breakdown.py "$@" > $O/$N.log 2>&1 || { tail -20 $O/$N.log; return 1; }
  grep calls $O/$N.log
  python3 tools/bins_timeline.py $O/$N.bin --skip 4 --show 2 > $O/${N}_tl.txt && cat $O/${N}_tl.txt
}
tl tl_one --frames 1 --calls 24 --warm 4 &&
tl tl_g16 --frames 16 --calls 8 --warm 4 &&
tl tl_share8_g16 --frames 16 --calls 8 --warm 4 --share 0/8 &&
tl tl_share8_g1 --frames 1 --calls 16 --warm 4 --share 0/8
