# Round-4 check + headline A/B: bash tools/gpu_r04b.sh TAG ROUNDS VARIANT... (after gpu_r04.sh's steps)
set -u
T=$1; N=$2; shift 2
bash tools/gpu_r04.sh $T "" --gpus 1 --steps 20 --warmup 5 || exit 1
bash tools/gpu_hab2.sh ${T}_ab $N "$@"
