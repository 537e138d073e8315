#!/bin/bash
# rocprofv3 kernel statistics of one bench command per library build (SAT_HIP_LIB_TUNING; "" = the product library),
# for a per-kernel A/B of two builds.   tools/prof_libs.sh TAG "BENCH ARGS" LIB [LIB...]
set -u
TAG=$1; ARGS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in "$@"; do
  name=${lib:-product}
  if [ -n "$lib" ]; then export SAT_HIP_LIB_TUNING=show-attend-and-tell_amd/libsat_hip_$lib.so; else unset SAT_HIP_LIB_TUNING; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$name" -o run --output-format csv -- \
      python bench.py --steps 60 --no-cpu-baseline --fp32-steps 0 --no-diagnostics $ARGS > "$OUT/prof_$name.log" 2>&1
  rc=$?
  echo "[$name] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
