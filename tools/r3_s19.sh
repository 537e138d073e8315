set -u
OUT=gpurun_out/r3_s19; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention or decoder or production" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
ab() {  # label, args...
  local label=$1; shift; i=$((i+1))
  timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --fp32-steps 0 --no-diagnostics "$@" > $OUT/ab_$i.log 2>&1 || { tail -5 $OUT/ab_$i.log; exit 1; }
  echo "[$label] $(python -c "import json,sys; d=json.loads([l for l in open('$OUT/ab_$i.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"
}
i=0
for r in 1 2; do
ab "cfg2"
ab "cfg2 fwd8" --policy attn_fwd=3
ab "cfg2 B64" --batch 64
ab "cfg2 B64 fwd8" --batch 64 --policy attn_fwd=3
done
timeout -k 10 300 env B=128 CONFIGS="1:0,0,0,0;1:0,0,0,0:3:0" python tools/bench_decoder_splits.py > $OUT/splits128.log 2>&1; grep -v amdgpu $OUT/splits128.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 2 --dist-backend gloo --no-cpu-baseline --fp32-steps 0 > $OUT/dp2_gloo.log 2>&1 || { tail -20 $OUT/dp2_gloo.log; exit 1; }
grep "^{" $OUT/dp2_gloo.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('dp2 gloo', d['value'], d['ms_per_step'], d['n_gpus'], d['config']['parallelism'], d['loss'])"
