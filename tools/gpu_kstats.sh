# kernel stats of tools/time_render.py (default library): bash tools/gpu_kstats.sh TAG [ENV...]
set -u
T=$1; shift
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T} -o k --output-format csv -- \
    python3 $R/tools/time_render.py --frames 20 > $R/gpurun_out/prof_${T}.log 2>&1 || exit 1
python3 - <<PY
import csv
for r in csv.DictReader(open("$R/gpurun_out/prof_${T}/k_kernel_stats.csv")):
    print(r['Name'][:70].ljust(70), r['Calls'].rjust(5), '%.4f' % (float(r['AverageNs']) / 1e6))
PY
