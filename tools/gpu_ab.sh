# A/B: default library vs variants, alternating, each run a fresh process.
# usage: bash tools/gpu_ab.sh TAG ROUNDS VARIANT...
set -u
T=$1; R=$2; shift 2
export TMPDIR=/tmp
for i in $(seq 1 $R); do
  for v in default "$@"; do
    L=""; [ $v != default ] && L=bih-gpu-raytracer_amd/lib/variants/libbih_amd_$v.so
    BIH_LIB=$L timeout -k 10 120 python tools/ab_group.py >> gpurun_out/${T}_ab.jsonl 2>/dev/null || exit 1
  done
done
python - <<PY
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/${T}_ab.jsonl"):
    j = json.loads(l); d[j["lib"]].append((j["ms_per_frame"], j["kernel_ms_per_frame"], j["img_hash"]))
for k, v in d.items():
    print(k, "ms/frame", sorted(round(x[0], 4) for x in v), "kernel/frame", sorted(round(x[1], 4) for x in v), "hash", set(x[2] for x in v))
PY
