# bench A/B of the overlap schedule knobs (no diagnostics); usage: bash tools/prio_ab.sh [args...]
set -e
for a in "$@"; do
  echo "== $a"
  timeout -k 10 120 python bench.py --steps 100 --no-cpu-baseline --fp32-steps 0 --no-diagnostics --enc-split none $a 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['encoder_trunk'].get('graph_ms_per_step'))"
done
