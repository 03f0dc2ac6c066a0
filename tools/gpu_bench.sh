# Round bench + profile (one GPU call): bench.py line, then the rocprofv3
# kernel-trace/stats summary of the same bench command (PMC traffic is
# measured by bench.py itself in child passes; disabled under the tracer).
set -u
TAG=$1
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
echo bench_rc=$rc; cat gpurun_out/bench_$TAG.json
[ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench_$TAG -o bench --output-format csv -- python3 $R/bench.py --traffic 0 --cpu-baseline 0 > $R/gpurun_out/bench_prof_$TAG.json 2>&1
echo prof_rc=$?
# isolated launches (one frame in flight) of the headline workload: their
# kernel average is the bench line's roofline.launch_ms
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_head_$TAG -o head --output-format csv -- python3 $R/bench.py --traffic 0 --cpu-baseline 0 --headline-only --in-flight 1 > $R/gpurun_out/bench_head_$TAG.json 2>&1
echo head_rc=$?
