#!/bin/bash
# Build an A/B variant library: the current objects with the given source files recompiled
# with extra defines.  usage: tools/build_def.sh <name> "<-Dflags>" <file.hip>...  ->
# t-vq-vae-trajgen_amd/lib_ab/libtvq_hip_<name>.so
set -e
name=$1; defs=$2; shift 2
cd "$(dirname "$0")/../t-vq-vae-trajgen_amd/csrc"
make -s -j8
mkdir -p build_ab_$name ../lib_ab
objs=""
for o in build/*.o; do
  b=$(basename $o .o)
  use=$o
  for f in "$@"; do
    if [ "$(basename $f .hip)" = "$b" ]; then
      /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I. -I../../include $defs -c $f -o build_ab_$name/$b.o
      use=build_ab_$name/$b.o
    fi
  done
  objs="$objs $use"
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../lib_ab/libtvq_hip_$name.so $objs
echo ../lib_ab/libtvq_hip_$name.so
