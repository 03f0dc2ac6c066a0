# kernel stats of the headline (isolated launches) + skip-trace timing
set -u
T=$1
R=$GRAFT_REPO_ROOT
J=gpurun_out/${T}_time.jsonl; rm -f $J
timeout -k 10 120 python tools/time_render.py --tag default >> $J 2>/dev/null || exit 1
BIH_LIB=bih-gpu-raytracer_amd/lib/variants/libbih_amd_skiptrace.so timeout -k 10 120 python tools/time_render.py --tag skiptrace >> $J 2>/dev/null || exit 1
grep -o '"tag[^,]*\|"ms_mean[^,]*' $J
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T} -o k --output-format csv -- \
    python3 $R/bench.py --headline-only --in-flight 1 --traffic 0 --cpu-baseline 0 --steps 50 > $R/gpurun_out/prof_${T}.log 2>&1 || exit 1
cut -d, -f1-4 $R/gpurun_out/prof_${T}/k_kernel_stats.csv | head -8 | cut -c1-150
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_if3 -o k --output-format csv -- \
    python3 $R/bench.py --headline-only --in-flight 3 --traffic 0 --cpu-baseline 0 --steps 50 > $R/gpurun_out/prof_${T}_if3.log 2>&1 || exit 1
cut -d, -f1-4 $R/gpurun_out/prof_${T}_if3/k_kernel_stats.csv | head -8 | cut -c1-150
