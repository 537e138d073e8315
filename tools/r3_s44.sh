set -u
OUT=gpurun_out/r3_s44; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "conv3x3_frag or vgg19_block5" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
ab() {  # label, args...
  local label=$1; shift; i=$((i+1))
  timeout -k 10 300 python bench.py --bert --network vgg19 --steps 60 --no-cpu-baseline --fp32-steps 0 "$@" > $OUT/ab_$i.log 2>&1 || { tail -5 $OUT/ab_$i.log; exit 1; }
  echo "[$label] $(python -c "import json,sys; d=json.loads([l for l in open('$OUT/ab_$i.log') if l.startswith('{')][-1]); t=d['encoder_trunk']; print(d['value'], d['ms_per_step'], 'trunk', t['conv_us_per_forward'], [ (k.split()[0],v['us']) for k,v in t['classes'].items() if k.split()[0] in ('conv1','conv4')])")"
}
i=0
for r in 1 2; do
ab "cfg5"
ab "cfg5 no112/224" --c2-frag-sizes 7,14,28
done
