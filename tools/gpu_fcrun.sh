set -u
R=$GRAFT_REPO_ROOT
for v in ${FCV:-fchead fcnolds fclds}; do
  echo "== $v"
  BIH_LIB=$R/bih-gpu-raytracer_amd/lib/variants/libbih_amd_$v.so timeout -k 10 120 python3 $R/tools/fast_counters.py --frames 2 2>&1 | grep -v "^$" | tail -8 || exit 1
done
