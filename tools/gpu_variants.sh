# timing of the default library and of each variant: gpu_variants.sh TAG V1 V2 ...
# V = a library variant name (lib/variants/libbih_amd_V.so) or env:NAME=VALUE
set -u
T=$1; shift
J=gpurun_out/${T}_var.jsonl; rm -f $J
timeout -k 10 120 python tools/time_render.py --tag default --frames 20 >> $J 2>/dev/null || exit 1
for V in "$@"; do
  case $V in
    env:*) env ${V#env:} timeout -k 10 120 python tools/time_render.py --frames 20 --tag $V >> $J 2>/dev/null || exit 1 ;;
    *) BIH_LIB=bih-gpu-raytracer_amd/lib/variants/libbih_amd_$V.so timeout -k 10 120 python tools/time_render.py --frames 20 --tag $V >> $J 2>/dev/null || exit 1 ;;
  esac
done
timeout -k 10 120 python tools/time_render.py --tag default2 --frames 20 >> $J 2>/dev/null || exit 1
grep -o '"tag[^,]*\|"ms_mean[^,]*\|"ms_median[^,]*\|"img_hash[^,}]*' $J | paste - - - -
