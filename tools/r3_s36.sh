set -u
OUT=gpurun_out/r3_s36; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { grep -E "^FAILED|Error|assert" $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 150 --no-cpu-baseline --fp32-steps 0 --no-diagnostics > $OUT/ab_$r.log 2>&1 || { tail -5 $OUT/ab_$r.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('$OUT/ab_$r.log') if l.startswith('{')][-1]); print('[cfg2]', d['value'], d['ms_per_step'], 'enc', d['encoder_trunk']['graph_ms_per_step'], 'dec', d['decoder_graphs_ms_per_step'])"
done
