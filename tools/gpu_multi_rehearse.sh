# Rehearses bench.py's N>1 path on a one-GPU box: all ranks on cuda:0 over
# gloo (BIH_BENCH_SHARE_GPU=1).  usage: bash tools/gpu_multi_rehearse.sh TAG
set -u
T=$1
export BIH_BENCH_SHARE_GPU=1 TMPDIR=/tmp
for n in 2 4; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 200 --warmup 16 \
    > gpurun_out/${T}_n$n.json 2> gpurun_out/${T}_n$n.err || { tail -30 gpurun_out/${T}_n$n.err; exit 1; }
  echo "n=$n"; python tools/bench_summary.py gpurun_out/${T}_n$n.json | head -3
done
