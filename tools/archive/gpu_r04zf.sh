bash tools/gpu_wh_ab.sh r04zf whs64 whs128 whs256
