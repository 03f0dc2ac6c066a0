# Round 5: the ring jump-table test alone, then the whole GPU suite
set -u
T=${1:-r05ad}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ring_advance or frames_in_flight" --timeout 120 --timeout-method thread \
    > $O/pytest1.log 2>&1; tail -30 $O/pytest1.log | grep -E "passed|failed|Error|assert" | head
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1; tail -3 $O/pytest.log
