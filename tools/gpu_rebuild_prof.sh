# Kernel trace of bench.py's legs (headline + with_rebuild + moving_camera), then the
# with_rebuild step timeline.  usage: bash tools/gpu_rebuild_prof.sh TAG
set -u
T=$1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_rb -o k --output-format csv -- \
    python3 $R/bench.py --steps 40 --warmup 10 --traffic 0 --cpu-baseline 0 --no-reference-leg --c5 0 --whitted-frames 0 \
    > $R/gpurun_out/${T}_rb.log 2>&1 || { tail -20 $R/gpurun_out/${T}_rb.log; exit 1; }
python3 $R/tools/rebuild_timeline.py $R/gpurun_out/${T}_rb/k_kernel_trace.csv 2
