# k_rng_init time per variant (rocprofv3 kernel stats).  usage: bash tools/gpu_rng_variants.sh TAG
set -u
T=$1
export TMPDIR=/tmp
for v in default run4 run32 run64; do
  L=""; [ $v != default ] && L=bih-gpu-raytracer_amd/lib/variants/libbih_amd_$v.so
  BIH_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_$v -o run -- python tools/time_rng.py --n 10 > gpurun_out/${T}_$v.log 2>&1 || { tail -5 gpurun_out/${T}_$v.log; exit 1; }
  python3 -c "import csv; print('$v', [(r['Calls'], float(r['AverageNs'])/1e3) for r in csv.DictReader(open('gpurun_out/${T}_$v/run_kernel_stats.csv')) if 'k_rng_init' in r['Name']])"
done
