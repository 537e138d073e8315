set -u
OUT=gpurun_out/r3_s55; mkdir -p $OUT; export TMPDIR=/tmp
ab() {  # label, args...
  local label=$1; shift; i=$((i+1))
  timeout -k 10 200 python bench.py --steps 150 --no-cpu-baseline --fp32-steps 0 --no-diagnostics "$@" > $OUT/ab_$i.log 2>&1 || { tail -5 $OUT/ab_$i.log; exit 1; }
  echo "[$label] $(python -c "import json,sys; d=json.loads([l for l in open('$OUT/ab_$i.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"
}
i=0
for r in 1 2 3; do
ab "cfg2"
ab "cfg2 slices2" --conv-slices 2
ab "cfg2 fb4" --feature-buffers 4
done
