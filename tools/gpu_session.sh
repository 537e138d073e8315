#!/bin/bash
# One GPU-box session: parity tests, conv A/B, graph bench, kernel-trace profile, PMC traffic passes.
# Every GPU step has its own time limit; the script stops at the first failing GPU step.
# usage: bash tools/gpu_session.sh TAG [steps...]   steps: tests bench prof pmc smoke
set -u
TAG=${1:-run}; shift
STEPS=${*:-"tests bench prof"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] $name: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  tail -4 "$OUT/$name.log"
  return $rc
}
for s in $STEPS; do
  case $s in
    tests) run tests 900 python -u -m pytest tests -m gpu -q --maxfail=30 -p no:cacheprovider --timeout 300 --timeout-method thread
           rc=$?; grep -E "^FAILED" "$OUT/tests.log" | head -30; [ $rc -le 1 ] || exit $rc ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 400 python bench.py || exit $? ;;
    benchno) run benchno 300 python bench.py --steps 50 --no-overlap --no-cpu-baseline --fp32-steps 0 || exit $? ;;
    benchq) run benchq 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit $? ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
               python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-graph || exit $? ;;
    profg) run profg 600 rocprofv3 --kernel-trace --stats -d "$OUT/profg" -o run --output-format csv -- \
               python bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit $? ;;
    pmc)   run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv -- \
               python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-graph || exit $?
           run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv -- \
               python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-graph || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
