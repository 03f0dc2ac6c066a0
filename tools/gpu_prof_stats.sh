# per-kernel device time of the bench workload (rocprofv3 kernel trace + stats)
set -u
T=$1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o k --output-format csv -- python3 $R/tools/prof_render.py --frames 20 > $R/gpurun_out/prof_$T.log 2>&1; echo prof=$?
f=$(find $R/gpurun_out/prof_$T -name '*kernel_stats.csv' | head -1)
cut -d, -f1-8 "$f" | head -20
