# effective clock of the render kernel: GRBM_GUI_ACTIVE (summed over the 8
# XCDs) / 8 / kernel time (MI355X_MICROARCH.md, DVFS give-back)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_clock
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d "$OUT/grbm" -o grbm --output-format csv -- \
    python3 "$R/tools/prof_render.py" --frames 5 > "$OUT/grbm.log" 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- \
    python3 "$R/tools/prof_render.py" --frames 5 > "$OUT/trace.log" 2>&1 || exit 1
python3 "$R/tools/summarize_prof.py" "$OUT"
