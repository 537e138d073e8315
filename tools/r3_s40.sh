set -u
OUT=gpurun_out/r3_s40; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "conv3x3_frag" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do timeout -k 10 200 python tools/conv_class_ab.py 64 --only L3c2 >> $OUT/conv_ab64.log 2>&1 || exit 1; done
cut -c1-1300 $OUT/conv_ab64.log | grep L3c2
ab() {  # label, args...
  local label=$1; shift; i=$((i+1))
  timeout -k 10 200 python bench.py --steps 150 --no-cpu-baseline --fp32-steps 0 --no-diagnostics "$@" > $OUT/ab_$i.log 2>&1 || { tail -5 $OUT/ab_$i.log; exit 1; }
  echo "[$label] $(python -c "import json,sys; d=json.loads([l for l in open('$OUT/ab_$i.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"
}
i=0
for r in 1 2; do
ab "B64" --batch 64
ab "B64 slices4" --batch 64 --conv-slices 3
done
