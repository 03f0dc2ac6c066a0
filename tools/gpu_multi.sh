# N=2 rehearsal of the distributed bench on one GPU (both ranks on cuda:0, gloo)
set -u
export BIH_BENCH_SHARE_GPU=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 2 --steps 40 --warmup 5 --traffic 0 --cpu-baseline 0 > gpurun_out/multi2.json 2> gpurun_out/multi2.err || { tail -20 gpurun_out/multi2.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/multi2.json').read().strip().splitlines()[-1]);print({k:d[k] for k in ('value','ms_per_step','n_gpus','scaling')}, 'side', json.dumps(d.get('other_decomposition'))[:300])"
