# kernel stats of the moving-camera workload (tools/prof_camera.py)
set -u
T=$1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T} -o k --output-format csv -- \
    python3 $R/tools/prof_camera.py --frames 16 > $R/gpurun_out/prof_${T}.log 2>&1 || exit 1
python3 - <<PY
import csv
for r in csv.DictReader(open("$R/gpurun_out/prof_${T}/k_kernel_stats.csv")):
    print(r['Name'][:60].ljust(60), r['Calls'].rjust(5), '%.4f' % (float(r['AverageNs']) / 1e6), '%.3f' % (float(r['TotalDurationNs']) / 1e6))
PY
