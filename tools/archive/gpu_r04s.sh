bash tools/gpu_wh_ab.sh r04s pfl10 pfl12 pfl16
