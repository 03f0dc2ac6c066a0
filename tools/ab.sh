# usage: bash tools/ab.sh TAG [variant libs...]: GPU tests, timings of the
# default library (anyhit + reference) and of each variant (anyhit), then the
# SQ instruction counters of the default library.
set -u
TAG=$1; shift
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout=300 -x > gpurun_out/t_$TAG.log 2>&1; rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/t_$TAG.log
[ $rc -eq 0 ] || exit 1
J=gpurun_out/ab_$TAG.jsonl; rm -f $J
for T in anyhit reference; do
  timeout -k 10 120 python tools/time_render.py --traverse $T --tag default >> $J 2>>gpurun_out/ab_$TAG.err || { echo "fail default $T"; exit 1; }
done
for V in "$@"; do
  BIH_LIB=bih-gpu-raytracer_amd/lib/variants/libbih_amd_$V.so timeout -k 10 120 python tools/time_render.py --traverse anyhit --tag "$V" >> $J 2>>gpurun_out/ab_$TAG.err || { echo "fail $V"; exit 1; }
done
cut -c1-200 $J
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/prof_$TAG/sq -o sq --output-format csv -- python3 $R/tools/prof_render.py --frames 3 > $R/gpurun_out/prof_$TAG.log 2>&1; echo sq_rc=$?
