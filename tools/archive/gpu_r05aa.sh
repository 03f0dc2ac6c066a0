# Round 5: advance with each thread's pixels loaded together and b128 table
# reads -- tests, A/B against HEAD, advance durations.
set -u
T=${1:-r05aa}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --durations=5 --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab5.sh $T 2 base hd || exit 1
cd /tmp && export TMPDIR=/tmp
for X in base hd; do
  L=""; [ $X = hd ] && L=$R/bih-gpu-raytracer_amd/lib/variants/libbih_amd_hd.so
  BIH_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/g16_$X -o k --output-format csv -- \
      python3 $R/tools/call_breakdown.py --frames 16 --calls 12 --sync 1 --streams 3 > $O/g16_$X.log 2>&1 || exit 1
  grep -h "k_rng_advance" $O/g16_$X/k_kernel_stats.csv | cut -d, -f1-4 | sed "s/^/$X /"
done
