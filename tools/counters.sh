#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group, --kernel-trace only) over single conv
# shapes.  usage: bash tools/counters.sh OUTDIR shape [shape...]
set -u
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
G2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INST_LEVEL_VMEM"
G3="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"
for shape in "$@"; do
  i=0
  for G in "$G1" "$G2" "$G3"; do
    i=$((i + 1))
    timeout -k 10 300 rocprofv3 --pmc $G --kernel-trace -d "$OUT/${shape}_$i" -o run --output-format csv -- \
      python tools/conv_one.py "$shape" 10 > "$OUT/${shape}_$i.log" 2>&1
    rc=$?
    echo "$shape group $i rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
