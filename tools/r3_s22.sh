set -u
OUT=gpurun_out/r3_s22; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "bottleneck_fused or encoder_fused or c2_frag_equal" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 200 python tools/block_ab.py 128 64 > $OUT/block_ab.log 2>&1 || { tail -20 $OUT/block_ab.log; exit 1; }
cat $OUT/block_ab.log
ab() {  # label, args...
  local label=$1; shift; i=$((i+1))
  timeout -k 10 200 python bench.py --steps 150 --no-cpu-baseline --fp32-steps 0 --no-diagnostics "$@" > $OUT/ab_$i.log 2>&1 || { tail -5 $OUT/ab_$i.log; exit 1; }
  echo "[$label] $(python -c "import json,sys; d=json.loads([l for l in open('$OUT/ab_$i.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"
}
i=0
for r in 1 2; do
ab "cfg2 L2 fused"
ab "cfg2 L2 unfused" --no-fuse-layer2
ab "B64 L2 fused" --batch 64
ab "B64 L2 unfused" --batch 64 --no-fuse-layer2
done
