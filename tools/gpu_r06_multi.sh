#!/bin/bash
# Round 6: bench.py's N > 1 path on a one-GPU box (ranks share cuda:0 over
# gloo, BIH_BENCH_SHARE_GPU=1) with the driver's default steps -- through the
# launcher (--gpus 2) and torch.distributed.run (4 ranks) -- and the band
# share projection of a long frame loop.  usage: tools/gpu_r06_multi.sh TAG
set -u
T=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
export TMPDIR=/tmp
BIH_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 > $O/n2.json 2> $O/n2.err || { tail -30 $O/n2.err; exit 1; }
BIH_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 4 --c5 0 > $O/n4.json 2> $O/n4.err || { tail -30 $O/n4.err; exit 1; }
timeout -k 10 400 python bench.py --steps 200 --warmup 16 --c5 1 --whitted-frames 0 --cpu-baseline 0 --traffic 0 \
  --host-loop 0 --no-reference-leg > $O/n1_steps200.json 2> $O/n1_steps200.err || { tail -30 $O/n1_steps200.err; exit 1; }
echo done
