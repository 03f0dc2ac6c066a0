set -u
bash tools/gpu_wh_ab.sh r04r whnp pf7 pfl6
