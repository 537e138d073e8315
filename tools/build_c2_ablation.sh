#!/bin/bash
# Diagnostics builds of the library for tools/c2_ablation.py: convblock.hip with SAT_C2_ABL = each given value,
# linked with the product objects into show-attend-and-tell_amd/libsat_hip_abl<N>.so (never loaded by the product).
set -eu
cd "$(dirname "$0")/../show-attend-and-tell_amd/csrc"
make -s -j8
for n in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DSAT_C2_ABL=$n -c convblock.hip -o build/convblock_abl$n.o
  objs=$(ls build/*.o | grep -v convblock | grep -v _abl | grep -v _v_)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libsat_hip_abl$n.so $objs build/convblock_abl$n.o
done
