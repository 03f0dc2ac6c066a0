#!/bin/bash
# Round 6 A/B of library variants on the driver's bench command (headline,
# window kernel time, one-frame, camera, rebuild, band share, C2):
# bash tools/gpu_ab6.sh TAG ROUNDS VARIANT...  (base = the in-tree library;
# VARIANT+ENV=1,ENV2=0 adds environment variables)
set -u
T=$1; N=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
V=$R/bih-gpu-raytracer_amd/lib/variants
for k in $(seq 1 $N); do
  for X in "$@"; do
    B=${X%%+*}; E=""; [ "$B" != "$X" ] && E=${X#*+}; E=${E//,/ }
    L=""; [ $B != base ] && L=$V/libbih_amd_$B.so
    env $E BIH_LIB=$L timeout -k 10 300 python -u bench.py --c5 0 --whitted-frames 0 --cpu-baseline 0 --traffic 0 \
        --no-reference-leg --host-loop 0 ${AB_ARGS:-} > $O/bench_${X}_$k.json 2> $O/bench_${X}_$k.err || { tail -20 $O/bench_${X}_$k.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w=d['roofline'].get('window') or {}
g=lambda k: (d.get(k) or {}).get('ms_per_step', float('nan'))
print(sys.argv[2], 'head %.4f' % d['ms_per_step'], 'wk %.4f' % w.get('kernel_ms_per_frame', float('nan')), 'launch %.4f' % (d['roofline']['launch_ms']/16), 'one %.4f' % g('one_in_flight'), 'cam %.4f' % g('moving_camera'), 'rb %.4f' % g('with_rebuild'), 'dyn %.4f' % g('dynamic_rebuild'), 'share %.3f' % d['band_share']['projected_efficiency'], 'c2 %.4f' % g('c2_torus'), 'eq', d.get('timed_outputs_equal'))
" $O/bench_${X}_$k.json $X | tee -a $O/ab.txt
  done
done
