#!/bin/bash
# Diagnostics build of the library with extra compile flags for some sources:
#   tools/build_variant.sh NAME "FLAGS" src.hip [src.hip...]  ->  show-attend-and-tell_amd/libsat_hip_NAME.so
# The product never loads it; A/B runs select it with SAT_HIP_LIB_TUNING (tools/session.sh abl:...).
set -eu
name=$1; flags=$2; shift 2
cd "$(dirname "$0")/../show-attend-and-tell_amd/csrc"
make -s -j8
objs=""
srcs=$(sed -n 's/^SRCS := //p' Makefile)
for f in build/*.o; do
  case $f in *_v_*) continue ;; esac
  case " $srcs " in *" $(basename "$f" .o).hip "*) ;; *) continue ;; esac   # stale objects of removed sources
  b=$(basename "$f" .o)
  skip=0
  for src in "$@"; do [ "$b" = "$(basename "$src" .hip)" ] && skip=1; done
  [ $skip = 1 ] || objs="$objs $f"
done
for src in "$@"; do
  b=$(basename "$src" .hip)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c "$src" -o "build/${b}_v_$name.o"
  objs="$objs build/${b}_v_$name.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "../libsat_hip_$name.so" $objs \
  -Wl,-rpath,/opt/rocm/lib
echo "built show-attend-and-tell_amd/libsat_hip_$name.so"
