set -u
OUT=gpurun_out/r3_s49; mkdir -p $OUT; export TMPDIR=/tmp
ab() {  # label, args...
  local label=$1; shift; i=$((i+1))
  timeout -k 10 200 python bench.py --steps 150 --no-cpu-baseline --fp32-steps 0 --no-diagnostics "$@" > $OUT/ab_$i.log 2>&1 || { tail -5 $OUT/ab_$i.log; exit 1; }
  echo "[$label] $(python -c "import json,sys; d=json.loads([l for l in open('$OUT/ab_$i.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], 'enc', d['encoder_trunk']['graph_ms_per_step'], 'dec', d['decoder_graphs_ms_per_step'])")"
}
i=0
for r in 1 2; do
ab "cfg2"
ab "cfg2 g2" --policy decoder_splits=0.0.2.0
ab "cfg2 g8" --policy decoder_splits=0.0.8.0
ab "cfg2 dh1" --policy decoder_splits=0.0.0.1
ab "cfg2 dh4" --policy decoder_splits=0.0.0.4
done
for r in 1 2; do
ab "B64"  --batch 64
ab "B64 nl2" --batch 64 --policy attn_bwd_chunks=2
ab "B64 split48" --batch 64 --split-target 48
ab "B64 split32" --batch 64 --split-target 32
done
