# Per-launch kernel trace of config C4 (k_wh_trace per bounce), 2 frames.
# usage: bash tools/gpu_wh_trace.sh TAG
set -u
T=$1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/${T}_wh -o k --output-format csv -- \
    python3 $R/tools/time_whitted.py --frames 1 > $R/gpurun_out/${T}_wh.log 2>&1 || exit 1
python3 - <<PY
import csv
rows = [r for r in csv.DictReader(open("$R/gpurun_out/${T}_wh/k_kernel_trace.csv")) if 'k_wh_' in r['Kernel_Name']]
for r in rows:
    print(r['Kernel_Name'][:40].ljust(40), '%.3f ms' % ((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6))
PY
