#!/bin/bash
# Builds libbih_amd from the sources of git revision REV (default HEAD) as a
# variant for A/B timing: tools/build_rev_variant.sh NAME [REV] ["DEFINES"]
# (REV "WORK" = the working tree) -> bih-gpu-raytracer_amd/lib/variants/libbih_amd_NAME.so
set -e
NAME=$1; REV=${2:-HEAD}; DEFS=${3:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/a/csrc $T/include $T/a/build
if [ "$REV" = WORK ]; then
  cp "$ROOT"/bih-gpu-raytracer_amd/csrc/* $T/a/csrc/
  cp "$ROOT"/include/bih.h $T/include/bih.h
else
  for f in $(git -C "$ROOT" ls-tree --name-only $REV bih-gpu-raytracer_amd/csrc/); do
    git -C "$ROOT" show $REV:$f > $T/a/csrc/$(basename $f)
  done
  git -C "$ROOT" show $REV:include/bih.h > $T/include/bih.h
fi
cd $T/a
for f in csrc/*.hip csrc/*.cpp; do
  b=$(basename $f)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize \
    -fno-gpu-rdc $DEFS -x hip -c $f -o build/$b.o &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
mkdir -p "$ROOT/bih-gpu-raytracer_amd/lib/variants"
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o "$ROOT/bih-gpu-raytracer_amd/lib/variants/libbih_amd_$NAME.so" build/*.o
rm -rf $T
