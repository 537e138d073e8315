set -u
OUT=gpurun_out/r3_s30; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { grep -E "^FAILED|Error" $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
ab() {  # label, args...
  local label=$1; shift; i=$((i+1))
  timeout -k 10 200 python bench.py --steps 150 --no-cpu-baseline --fp32-steps 0 --no-diagnostics "$@" > $OUT/ab_$i.log 2>&1 || { tail -5 $OUT/ab_$i.log; exit 1; }
  echo "[$label] $(python -c "import json,sys; d=json.loads([l for l in open('$OUT/ab_$i.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['encoder_trunk']['graph_ms_per_step'])")"
}
i=0
for r in 1 2 3; do
ab "cfg2"
ab "cfg2 enc-first" --enqueue encoder-first
done
ab "B64"  --batch 64
ab "B64 enc-first" --batch 64 --enqueue encoder-first
