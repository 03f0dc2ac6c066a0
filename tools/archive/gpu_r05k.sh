# Round 5: call shapes for the driver's 20 steps (--group 16 / 20 / 64) and a
# kernel trace of the driver command's timed region.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05k
mkdir -p $O
cd $R
for k in 1 2; do
  for G in 16 20 64; do
    timeout -k 10 300 python -u bench.py --group $G --headline-only --cpu-baseline 0 --traffic 0 \
        > $O/head_g${G}_$k.json 2> $O/head_g${G}_$k.err || { tail -20 $O/head_g${G}_$k.err; exit 1; }
    timeout -k 10 300 python -u bench.py --group $G --steps 500 --warmup 50 --headline-only --cpu-baseline 0 --traffic 0 \
        > $O/head500_g${G}_$k.json 2> $O/head500_g${G}_$k.err || { tail -20 $O/head500_g${G}_$k.err; exit 1; }
    python3 -c "
import json,sys
a=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); b=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print('group', sys.argv[3], '20 steps %.4f ms/frame' % a['ms_per_step'], 'launch %.4f' % (a['roofline']['launch_ms']/int(sys.argv[3])), '| 500 steps %.4f' % b['ms_per_step'])
" $O/head_g${G}_$k.json $O/head500_g${G}_$k.json $G | tee -a $O/ab.txt
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_head -o k --output-format csv -- \
    python3 $R/bench.py --headline-only --cpu-baseline 0 --traffic 0 --kernel-samples 0 > $O/trace_head.log 2>&1 || exit 1
python3 - $O/trace_head/k_kernel_trace.csv <<'PY' | tee $O/trace_head_tail.txt
import csv, re, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
def nm(r):
    m = re.search(r"(k_\w+|__amd\w+)", r["Kernel_Name"]); return m.group(1) if m else r["Kernel_Name"][:24]
tail = rows[-14:]
t0 = int(tail[0]["Start_Timestamp"])
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%-22s q%-3s start %9.1f dur %8.1f end %9.1f" % (nm(r), r["Queue_Id"], (s - t0) / 1e3, (e - s) / 1e3, (e - t0) / 1e3))
PY
