# Per-camera kernel times (rocprofv3 kernel trace of tools/prof_camera.py)
# for the tree's library and variants.  usage: bash tools/gpu_kcam_ab.sh TAG [VARIANT...]
set -u
T=$1; shift
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in default "$@"; do
  if [ $v = default ]; then L=""; else L="BIH_LIB=$R/bih-gpu-raytracer_amd/lib/variants/libbih_amd_$v.so"; fi
  env $L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_$v -o k --output-format csv -- \
      python3 $R/tools/prof_camera.py --frames 16 > $R/gpurun_out/${T}_$v.log 2>&1 || exit 1
  echo "== $v"
  python3 - <<PY
import csv
for r in csv.DictReader(open("$R/gpurun_out/${T}_$v/k_kernel_stats.csv")):
    if any(k in r['Name'] for k in ('k_bin_', 'k_cam_tris', 'k_render_bins')):
        print(r['Name'][:60].ljust(60), r['Calls'].rjust(5), '%.4f' % (float(r['AverageNs']) / 1e6))
PY
done
