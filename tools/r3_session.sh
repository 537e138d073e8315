#!/bin/bash
# One GPU-box session of round 3: full GPU suite, smoke, the default bench, a B = 64 line, and a
# rocprofv3 kernel trace of the default bench command (summarised by tools/prof_summary.py).
# usage: bash tools/r3_session.sh TAG [steps...]   steps: tests smoke bench bench64 prof
set -u
TAG=${1:-r3}; shift
STEPS=${*:-"tests smoke bench bench64 prof"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] $name: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  tail -3 "$OUT/$name.log" | cut -c1-400
  return $rc
}
for s in $STEPS; do
  case $s in
    tests) run tests 900 python -u -m pytest tests -m gpu -q --maxfail=20 -p no:cacheprovider --timeout 300 --timeout-method thread
           rc=$?; grep -E "^FAILED" "$OUT/tests.log" | head -30; [ $rc -le 1 ] || exit $rc ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 400 python bench.py || exit $? ;;
    bench64) run bench64 300 python bench.py --batch 64 --no-cpu-baseline --fp32-steps 0 || exit $? ;;
    benchq) run benchq 300 python bench.py --steps 100 --no-cpu-baseline --fp32-steps 0 || exit $? ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
               python bench.py || exit $?
           python tools/prof_summary.py "$OUT/prof" "$OUT/prof.log" "$OUT/prof_summary.json" | head -60 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
