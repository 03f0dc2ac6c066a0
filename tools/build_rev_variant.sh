#!/bin/bash
# Builds libbih_amd from the sources of git revision REV (default HEAD) as a
# variant for A/B timing: tools/build_rev_variant.sh NAME [REV] ["DEFINES"]
# -> bih-gpu-raytracer_amd/lib/variants/libbih_amd_NAME.so
set -e
NAME=$1; REV=${2:-HEAD}; DEFS=${3:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/a/csrc $T/include $T/a/build
for f in bih_build.hip bih_render.hip bih_capi.cpp xorwow_host.cpp bih_obj.cpp bih_internal.h bih_packet_asm.h; do
  git -C "$ROOT" show $REV:bih-gpu-raytracer_amd/csrc/$f > $T/a/csrc/$f
done
git -C "$ROOT" show $REV:include/bih.h > $T/include/bih.h
cd $T/a
for f in bih_build.hip bih_render.hip bih_capi.cpp xorwow_host.cpp bih_obj.cpp; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize \
    -fno-gpu-rdc $DEFS -x hip -c csrc/$f -o build/$f.o &
done
wait
mkdir -p "$ROOT/bih-gpu-raytracer_amd/lib/variants"
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o "$ROOT/bih-gpu-raytracer_amd/lib/variants/libbih_amd_$NAME.so" build/*.o
rm -rf $T
