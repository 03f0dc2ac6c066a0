#!/bin/bash
# rocprofv3 passes over tools/prof_render.py (run on the GPU box).
# usage: tools/profile.sh <tag> [extra prof_render args]
# kernel trace + stats, then one --pmc pass per counter group (never combined
# with other tracing); outputs under gpurun_out/prof_<tag>/.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o "$name" --output-format csv -- \
      python3 "$R/tools/prof_render.py" "${PROF_ARGS[@]}" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
PROF_ARGS=("$@")
run trace --kernel-trace --stats || exit 1
run fetch --pmc FETCH_SIZE || exit 1
run write --pmc WRITE_SIZE || exit 1
run sq1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY || exit 1
run sq2 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_BRANCH || exit 1
run tcc --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum || exit 1
run sq3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_INSTS_SCRATCH || echo "sq3 (optional) failed"
echo all-done
