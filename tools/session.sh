#!/bin/bash
# One GPU-box session: every GPU step runs under its own time limit, the script stops at the first
# failing GPU step (no retries), and every log lands under gpurun_out/TAG/.
#
# usage: bash tools/session.sh TAG step [step...]
#   tests              the whole GPU suite (-m gpu)
#   tests:EXPR         GPU tests selected by -k EXPR
#   testsv:EXPR        the same with their output (-s), every selected test run
#   smoke              __graft_entry__.smoke()
#   bench              the default bench line (the driver's command)
#   bench64            the B = 64 line (cfg2 / cfg3's per-rank shape), no CPU baseline / fp32 leg
#   benchq             a quick B = 128 line (100 steps, no CPU baseline / fp32 leg)
#   cfg4 | cfg5        the --no-tf / --bert --network vgg19 lines
#   dpr                bench.py --dp-rehearse: the N > 1 path over a one-rank RCCL process group
#   gloo2              bench.py as two ranks over gloo on the one GPU at --batch 64 (the N > 1 path, cfg3 per rank)
#   prof               rocprofv3 --kernel-trace --stats of the default bench command (+ tools/prof_summary.py)
#   prof:LABEL:ARGS    the same over a quick bench line with extra flags (A/B of per-kernel times)
#   pmcdec             two PMC passes (FETCH_SIZE, WRITE_SIZE) over the decoder's per-step kernels
#                      (tools/decoder_pmc.py; summary -> gpurun_out/TAG/pmc_decoder.json)
#   pmctrunk           FETCH_SIZE / WRITE_SIZE passes over an eager bench: per conv class HBM bytes (pmc_traffic.py)
#   pmcdec2            SQ / TCC counter groups over the same decoder run (per-kernel means -> pmc2_*.json)
#   ab:LABEL:ARGS      one A/B bench line (ARGS comma-separated bench.py flags, e.g. ab:st80:--split-target,80);
#                      prints value and ms/step
#   abl:LABEL:LIB:ARGS the same with the diagnostics build show-attend-and-tell_amd/libsat_hip_LIB.so
#                      (tools/build_variant.sh) loaded instead of the product library
#   abd:LABEL:ARGS     the same with the diagnostics (per-step decoder kernels, trunk classes; tools/bench_brief.py)
#   abdl:LABEL:LIB:ARGS  abd with the diagnostics build libsat_hip_LIB.so
#   py:SCRIPT[:ARGS]   python SCRIPT ARGS (comma-separated) under a 300 s limit
set -u
TAG=${1:?tag}; shift
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
line() {  # value and ms/step of a bench log
  python - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(d["value"], d["ms_per_step"])
PY
}
QUIET="--no-cpu-baseline --fp32-steps 0"
n=0
for s in "$@"; do
  n=$((n + 1))
  case $s in
    tests) run tests 900 python -u -m pytest tests -m gpu -q --maxfail=20 -p no:cacheprovider --timeout 300 \
               --timeout-method thread
           rc=$?; grep -E "^FAILED" "$OUT/tests.log" | head -30; [ $rc -le 1 ] || exit $rc ;;
    tests:*) run tests_$n 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 \
               --timeout-method thread -k "${s#tests:}"
           rc=$?; grep -E "^FAILED" "$OUT/tests_$n.log" | head -30; [ $rc -le 1 ] || exit $rc ;;
    testsv:*) run testsv_$n 900 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 600 \
               --timeout-method thread -k "${s#testsv:}"
           rc=$?; grep -E "^FAILED|gradient errors" "$OUT/testsv_$n.log" | head -40; [ $rc -le 1 ] || exit $rc ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 400 python bench.py || exit $? ;;
    bench64) run bench64 300 python bench.py --batch 64 $QUIET || exit $? ;;
    benchq) run benchq 300 python bench.py --steps 100 $QUIET || exit $? ;;
    cfg4) run cfg4 300 python bench.py --no-tf $QUIET || exit $? ;;
    dpr)   # the data-parallel path of bench.py over a one-rank RCCL process group (--dp-rehearse)
      run dpr 300 python bench.py --dp-rehearse --steps 30 --no-cpu-baseline --fp32-steps 0 || exit $? ;;
    gloo2) # the N > 1 path rehearsed on one GPU: two ranks over gloo at cfg3's per-rank batch (64)
           # (bench.py --gpus 2 starts the two ranks itself, as the driver's `bench.py --gpus N` does)
           run gloo2 400 python bench.py --gpus 2 --batch 64 --dist-backend gloo --steps 30 $QUIET || exit $? ;;
    cfg5) run cfg5 300 python bench.py --bert --network vgg19 $QUIET || exit $? ;;
    prof:*) rest=${s#prof:}; label=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
          run prof_$label 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$label" -o run --output-format csv -- \
              python bench.py --steps 100 $QUIET --no-diagnostics ${args//,/ } || exit $?
          python tools/prof_summary.py "$OUT/prof_$label" "$OUT/prof_$label.log" "$OUT/prof_$label.json" | head -40 ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
              python bench.py || exit $?
          python tools/prof_summary.py "$OUT/prof" "$OUT/prof.log" "$OUT/prof_summary.json" | head -60 ;;
    pmcdec)
      for c in FETCH_SIZE WRITE_SIZE; do
        run pmc_$c 300 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc_$c" -o run --output-format csv -- \
            python tools/decoder_pmc.py || exit $?
      done
      python tools/decoder_pmc.py --analyze "$OUT/pmc_FETCH_SIZE" "$OUT/pmc_WRITE_SIZE" "$OUT/pmc_decoder.json" ;;
    pmctrunk)   # the encoder conv classes' HBM traffic (tools/pmc_traffic.py): eager bench, two passes
      for c in FETCH_SIZE WRITE_SIZE; do
        run pmct_$c 400 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmct_$c" -o run --output-format csv -- \
            python bench.py --no-graph --steps 3 --warmup 1 $QUIET --no-diagnostics || exit $?
      done
      python tools/pmc_traffic.py "$OUT/pmct_FETCH_SIZE" "$OUT/pmct_WRITE_SIZE" resnet152 128 \
          "$OUT/pmc_traffic_resnet152.json" | tail -30 ;;
    pmcdec2)   # SQ and TCC counter groups over the same decoder run (one rocprofv3 pass per group)
      i=0
      for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU" \
               "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
        i=$((i + 1))
        run pmc2_$i 300 rocprofv3 --pmc $G --kernel-trace -d "$OUT/pmc2_$i" -o run --output-format csv -- \
            python tools/decoder_pmc.py || exit $?
        python tools/decoder_pmc.py --counters "$OUT/pmc2_$i" "$OUT/pmc2_$i.json" | head -80
      done ;;
    ab:*) rest=${s#ab:}; label=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
          run ab_${n}_$label 300 python bench.py --steps 150 $QUIET --no-diagnostics ${args//,/ } || exit $?
          echo "[$label] $(line "$OUT/ab_${n}_$label.log")" ;;
    abl:*) rest=${s#abl:}; label=${rest%%:*}; rest=${rest#*:}; lib=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
          SAT_HIP_LIB_TUNING=show-attend-and-tell_amd/libsat_hip_$lib.so \
            run ab_${n}_$label 300 python bench.py --steps 150 $QUIET --no-diagnostics ${args//,/ } || exit $?
          echo "[$label] $(line "$OUT/ab_${n}_$label.log")" ;;
    abd:*) rest=${s#abd:}; label=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
          run abd_${n}_$label 300 python bench.py --steps 100 $QUIET ${args//,/ } || exit $?
          python tools/bench_brief.py "$OUT/abd_${n}_$label.log" ;;
    abdl:*) rest=${s#abdl:}; label=${rest%%:*}; rest=${rest#*:}; lib=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
          SAT_HIP_LIB_TUNING=show-attend-and-tell_amd/libsat_hip_$lib.so \
            run abd_${n}_$label 300 python bench.py --steps 100 $QUIET ${args//,/ } || exit $?
          python tools/bench_brief.py "$OUT/abd_${n}_$label.log" ;;
    py:*) rest=${s#py:}; script=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
          run py_${n}_$(basename "$script" .py) 300 python "$script" ${args//,/ } || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
