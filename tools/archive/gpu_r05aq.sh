# Round 5: the steady-loop allocation test with its single-stream (stamped) part
set -u
T=${1:-r05aq}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "allocates_nothing or stamped" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; tail -3 $O/pytest.log
