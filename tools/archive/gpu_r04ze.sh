set -u
bash tools/gpu_wh_ab.sh r04ze whs64 whr8 whr32 || exit 1
BIH_WH_SORT=0 timeout -k 10 300 python3 tools/time_whitted.py --frames 2 > gpurun_out/r04ze_nosort.json 2>/dev/null || exit 1
echo "== nosort $(tail -1 gpurun_out/r04ze_nosort.json | cut -c1-100)"
