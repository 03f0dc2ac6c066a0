#!/bin/bash
# Builds libbih_amd variants for A/B timing: tools/build_variants.sh NAME "DEFINES" [NAME "DEFINES" ...]
# -> bih-gpu-raytracer_amd/lib/variants/libbih_amd_NAME.so
set -e
cd "$(dirname "$0")/../bih-gpu-raytracer_amd"
while [ $# -ge 2 ]; do
  NAME=$1; DEFS=$2; shift 2
  mkdir -p lib/variants build/v_$NAME
  for f in bih_build.hip bih_render.hip bih_bins.hip bih_whitted.hip bih_capi.cpp xorwow_host.cpp bih_obj.cpp; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -fno-gpu-rdc \
      $DEFS -x hip -c csrc/$f -o build/v_$NAME/$f.o &
  done
  wait
  /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o lib/variants/libbih_amd_$NAME.so build/v_$NAME/*.o
done
