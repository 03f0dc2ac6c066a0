set -u
for cfg in "c3:" "c5:--tris 10000000 --width 3840 --height 2160"; do
  name=${cfg%%:*}; args=${cfg#*:}
  for f in 1 2 3; do
    timeout -k 10 300 python bench.py $args --headline-only --in-flight $f --steps 400 --warmup 40 --traffic 0 --cpu-baseline 0 > gpurun_out/r03v_${name}_f$f.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/r03v_${name}_f$f.json').read().splitlines()[-1]);print('$name in-flight $f', round(d['ms_per_step'],4), '%.4g'%d['value'])"
  done
done
