set -u
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for m in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r04v_r$m -o k --output-format csv -- \
    python3 $R/tools/time_host_rebuild.py --render $m > $R/gpurun_out/r04v_r$m.log 2>&1 || exit 1
  grep "host us" $R/gpurun_out/r04v_r$m.log
  python3 - <<PY
import csv
for r in csv.DictReader(open("$R/gpurun_out/r04v_r$m/k_kernel_stats.csv")):
    print('  ', r['Name'][:50].ljust(50), r['Calls'].rjust(5), '%.1f' % (float(r['AverageNs']) / 1e3))
PY
done
