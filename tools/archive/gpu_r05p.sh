# Round 5: per-dispatch PMC of isolated 16-frame k_render_bins launches (ring
# and stamped instances), SQ counters, the driver command's timed region.
set -u
T=${1:-r05p}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
pmc() {   # pmc NAME ENV COUNTERS
  local N=$1; local E=$2; local C=$3
  env $E timeout -s KILL 120 rocprofv3 --pmc $C -d $O/$N -o pmc --output-format csv -- \
      python3 $R/tools/call_breakdown.py --frames 16 --calls 8 --warm 4 --sync 1 > $O/$N.log 2>&1 || { tail -5 $O/$N.log; return 1; }
  python3 $R/tools/pmc_dispatch.py $O/$N > $O/${N}.txt; tail -3 $O/${N}.txt
}
pmc fetch_ring BIH_STAMPED=0 FETCH_SIZE &&
pmc write_ring BIH_STAMPED=0 WRITE_SIZE &&
pmc fetch_st BIH_STAMPED=1 FETCH_SIZE &&
pmc write_st BIH_STAMPED=1 WRITE_SIZE &&
pmc sq_ring BIH_STAMPED=0 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" || exit 1
# per-dispatch FETCH over the bench's own traffic driver (3 calls of 16 frames)
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_prof -o pmc --output-format csv -- \
    python3 $R/tools/prof_render.py --frames 6 --group 16 > $O/fetch_prof.log 2>&1 &&
python3 $R/tools/pmc_dispatch.py $O/fetch_prof > $O/fetch_prof.txt; cat $O/fetch_prof.txt
# the driver command's timed region: kernel trace, last two calls
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_head -o k --output-format csv -- \
    python3 $R/bench.py --headline-only --cpu-baseline 0 --traffic 0 --kernel-samples 0 > $O/trace_head.log 2>&1 || exit 1
grep '"value"' $O/trace_head.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('head', d['ms_per_step'])"
python3 - $O/trace_head/k_kernel_trace.csv <<'PY' | tee $O/trace_head_tail.txt
import csv, re, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
def nm(r):
    m = re.search(r"(k_\w+|__amd\w+)", r["Kernel_Name"]); return m.group(1) if m else r["Kernel_Name"][:24]
# from the third-last k_render_bins (the last warm-up call) on
idx = [i for i, r in enumerate(rows) if "k_render_bins" in r["Kernel_Name"]]
tail = rows[max(0, idx[-3] - 3):] if len(idx) >= 3 else rows[-20:]
t0 = int(tail[0]["Start_Timestamp"])
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%-22s q%-3s start %9.1f dur %8.1f end %9.1f" % (nm(r), r.get("Queue_Id", "?"), (s - t0) / 1e3, (e - s) / 1e3, (e - t0) / 1e3))
PY
