set -u
OUT=gpurun_out/r3_s15; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
B="python bench.py --steps 150 --no-cpu-baseline --fp32-steps 0 --no-diagnostics"
i=0
for v in "" "--policy attn_bwd_chunks=1" "--split-target 32" "--split-target 128" "--stream-priority equal" "--fuse-every 5" "--policy gemm_stages=3" ""; do
  i=$((i+1)); timeout -k 10 200 $B $v > $OUT/ab_$i.log 2>&1 || { tail -5 $OUT/ab_$i.log; exit 1; }
  echo "[$v] $(python -c "import json,sys; d=json.loads([l for l in open('$OUT/ab_$i.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 300 python bench.py --no-tf --steps 100 --no-cpu-baseline --fp32-steps 0 > $OUT/cfg4.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --bert --network vgg19 --steps 100 --fp32-steps 0 > $OUT/cfg5.log 2>&1 || exit 1
python tools/bench_brief.py $OUT/cfg4.log $OUT/cfg5.log | grep -v "^    [a-z]"
