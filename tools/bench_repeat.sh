# The driver's bench command three times in one session (run-to-run spread on one box, and its wall time).
set -u
O=gpurun_out/r5_s33; mkdir -p $O
for i in 1 2 3; do
  s=$(date +%s.%N)
  timeout -k 10 400 python bench.py > $O/bench_$i.log 2>&1 || exit $?
  e=$(date +%s.%N)
  python - $O/bench_$i.log $s $e <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[1], d["value"], d["ms_per_step"], "wall %.1f s" % (float(sys.argv[3]) - float(sys.argv[2])))
PY
done
