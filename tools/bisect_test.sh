#!/bin/bash
# Run one GPU test selection against the product library and diagnostics builds (SAT_HIP_LIB_TUNING), in turn;
# stops at the first run that ends other than pass / fail (a fault, abort or time limit).
#   tools/bisect_test.sh TAG "PYTEST -k EXPR" [LIB...]   (LIB: show-attend-and-tell_amd/libsat_hip_LIB.so; "" = product)
set -u
TAG=$1; EXPR=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for lib in "" "$@"; do
  name=${lib:-product}
  if [ -n "$lib" ]; then export SAT_HIP_LIB_TUNING=show-attend-and-tell_amd/libsat_hip_$lib.so; else unset SAT_HIP_LIB_TUNING; fi
  timeout -k 10 300 python -u -m pytest tests -m gpu -k "$EXPR" -x -q -p no:cacheprovider --timeout 120 \
      --timeout-method thread > "$OUT/$name.log" 2>&1
  rc=$?
  echo "[$name] rc=$rc $(tail -1 "$OUT/$name.log")"
  [ $rc -le 1 ] || exit $rc
done
