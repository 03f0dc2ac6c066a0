bash tools/gpu_wh_ab.sh r04zg whs256 whs512 whs1024
