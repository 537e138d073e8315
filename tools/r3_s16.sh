set -u
OUT=gpurun_out/r3_s16; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention or decoder or frag or skinny" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 150 --no-cpu-baseline --fp32-steps 0 --no-diagnostics"
i=0
for v in "" "--policy lstm_blocks=256" "--policy lstm_blocks=128" "--policy attn_bwd_chunks=2" ""; do
  i=$((i+1)); timeout -k 10 200 $B $v > $OUT/ab_$i.log 2>&1 || { tail -5 $OUT/ab_$i.log; exit 1; }
  echo "[$v] $(python -c "import json,sys; d=json.loads([l for l in open('$OUT/ab_$i.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"
done
for v in "" "--conv-slices 6" "--conv-slices 7"; do
  i=$((i+1)); timeout -k 10 200 $B --batch 64 $v > $OUT/ab_$i.log 2>&1 || { tail -5 $OUT/ab_$i.log; exit 1; }
  echo "[B64 $v] $(python -c "import json,sys; d=json.loads([l for l in open('$OUT/ab_$i.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 300 python bench.py --batch 64 --steps 100 --no-cpu-baseline --fp32-steps 0 --conv-slices 6 > $OUT/bench64_s6.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --batch 64 --steps 100 --no-cpu-baseline --fp32-steps 0 --conv-slices 7 > $OUT/bench64_s7.log 2>&1 || exit 1
python tools/bench_brief.py $OUT/bench64_s6.log $OUT/bench64_s7.log | grep -v "^    [a-z]"
timeout -k 10 300 python bench.py --no-tf --steps 100 --no-cpu-baseline --fp32-steps 0 > $OUT/cfg4.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --bert --network vgg19 --steps 100 --fp32-steps 0 > $OUT/cfg5.log 2>&1 || exit 1
python tools/bench_brief.py $OUT/cfg4.log $OUT/cfg5.log | grep -v "^    [a-z]"
