# kernel traces of the driver command's timed region at --group 16 and 20
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05l
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for G in 16 20; do
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_g$G -o k --output-format csv -- \
    python3 $R/bench.py --group $G --headline-only --cpu-baseline 0 --traffic 0 --kernel-samples 0 > $O/trace_g$G.log 2>&1 || exit 1
grep '"value"' $O/trace_g$G.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('G', $G, d['ms_per_step'])"
python3 - $O/trace_g$G/k_kernel_trace.csv <<'PY' | tee $O/trace_g${G}_tail.txt
import csv, re, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
def nm(r):
    m = re.search(r"(k_\w+|__amd\w+)", r["Kernel_Name"]); return m.group(1) if m else r["Kernel_Name"][:24]
tail = rows[-22:]
t0 = int(tail[0]["Start_Timestamp"])
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%-22s q%-3s start %9.1f dur %8.1f end %9.1f" % (nm(r), r["Queue_Id"], (s - t0) / 1e3, (e - s) / 1e3, (e - t0) / 1e3))
PY
done
