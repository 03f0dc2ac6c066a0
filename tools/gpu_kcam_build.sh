# Kernel stats of the moving-camera workload and of repeated rebuilds.
# usage: bash tools/gpu_kcam_build.sh TAG
set -u
T=$1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for w in camera build; do
  if [ $w = camera ]; then cmd="$R/tools/prof_camera.py --frames 16"; else cmd="$R/tools/prof_build.py --builds 10"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_$w -o k --output-format csv -- \
      python3 $cmd > $R/gpurun_out/${T}_$w.log 2>&1 || exit 1
  python3 - <<PY > $R/gpurun_out/${T}_$w.txt
import csv
for r in csv.DictReader(open("$R/gpurun_out/${T}_$w/k_kernel_stats.csv")):
    print(r['Name'][:60].ljust(60), r['Calls'].rjust(5), '%.4f' % (float(r['AverageNs']) / 1e6), '%.3f' % (float(r['TotalDurationNs']) / 1e6))
PY
  echo "== $w"; head -25 $R/gpurun_out/${T}_$w.txt
done
tail -2 $R/gpurun_out/${T}_build.log
