# Round 5: bench.py's N>1 path rehearsed on the one-GPU box (2 ranks on
# cuda:0 over gloo, the driver's step counts), with the final library.
set -u
T=${1:-r05ak}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
export BIH_BENCH_SHARE_GPU=1 TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --gpus 2 --steps 20 --warmup 5 > $O/n2.json 2> $O/n2.err || { tail -30 $O/n2.err; exit 1; }
tail -c 600 $O/n2.json; echo
