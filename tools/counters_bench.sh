#!/bin/bash
# PMC counter passes over one eager bench.py step (one rocprofv3 run per counter group).
# usage: bash tools/counters_bench.sh OUTDIR ; then KFILTER=<kernel substring> python tools/counters_summary.py OUTDIR
set -u
OUT=$1
export TMPDIR=/tmp
mkdir -p "$OUT"
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
G2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VALU"
G3="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for G in "$G1" "$G2" "$G3"; do
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --pmc $G --kernel-trace -d "$OUT/bench_$i" -o run --output-format csv -- \
    python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-graph > "$OUT/bench_$i.log" 2>&1
  rc=$?
  echo "group $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
