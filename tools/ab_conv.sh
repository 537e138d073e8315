# A/B of conv configs on the ResNet152 shapes: baseline library (tools/libsat_base.so) vs the in-tree one
set -e
export SHAPES=${SHAPES:-L1_c3,L2_c3,L3_c3,L3_c2,L3_c1} CONFIGS=${CONFIGS:-2,1,1}
for r in 1 2; do
  echo "== base $r"; SAT_HIP_LIB_TUNING=$PWD/tools/libsat_base.so timeout -k 10 120 python tools/bench_conv.py 2>&1 | grep -v amdgpu.ids
  [ -n "$BASE_ONLY" ] && continue
  echo "== new $r"; timeout -k 10 120 python tools/bench_conv.py 2>&1 | grep -v amdgpu.ids
done
