# Round 5: light tail items (the cheapest tiles split over short frame ranges) -- tests, A/B,
# kernel trace of the driver command's timed region and of isolated calls.
set -u
T=${1:-r05r}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --durations=5 --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab5.sh $T 2 base base+BIH_TAIL_FRAC=0 base+BIH_TAIL_FRAC=0.3 base+BIH_TAIL_FRAMES=2 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_head -o k --output-format csv -- \
    python3 $R/bench.py --headline-only --cpu-baseline 0 --traffic 0 --kernel-samples 0 > $O/trace_head.log 2>&1 || exit 1
grep '"value"' $O/trace_head.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('head', d['ms_per_step'])"
python3 - $O/trace_head/k_kernel_trace.csv <<'PY' | tee $O/trace_head_tail.txt
import csv, re, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
def nm(r):
    m = re.search(r"(k_\w+|__amd\w+)", r["Kernel_Name"]); return m.group(1) if m else r["Kernel_Name"][:24]
idx = [i for i, r in enumerate(rows) if "k_render_bins" in r["Kernel_Name"]]
tail = rows[max(0, idx[-3] - 3): idx[-1] + 2]
t0 = int(tail[0]["Start_Timestamp"])
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%-22s q%-3s start %9.1f dur %8.1f end %9.1f" % (nm(r), r.get("Queue_Id", "?"), (s - t0) / 1e3, (e - s) / 1e3, (e - t0) / 1e3))
PY
