#!/bin/bash
# Run one diagnostics script against the product library and diagnostics builds in turn (SAT_HIP_LIB_TUNING);
# stops at the first run that does not exit 0.
#   tools/py_libs.sh TAG SCRIPT "ARGS" [LIB...]   ("" = the product library)
set -u
TAG=$1; SCRIPT=$2; ARGS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for lib in "$@"; do
  name=${lib:-product}
  if [ -n "$lib" ]; then export SAT_HIP_LIB_TUNING=show-attend-and-tell_amd/libsat_hip_$lib.so; else unset SAT_HIP_LIB_TUNING; fi
  timeout -k 10 300 python -u "$SCRIPT" $ARGS > "$OUT/$(basename "$SCRIPT" .py)_$name.log" 2>&1
  rc=$?
  echo "[$name] rc=$rc"
  tail -4 "$OUT/$(basename "$SCRIPT" .py)_$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
