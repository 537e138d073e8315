set -u
OUT=gpurun_out/r3_s18; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; grep -E "^FAILED|Error" $OUT/tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
timeout -k 10 300 python bench.py --batch 64 --no-cpu-baseline --fp32-steps 0 > $OUT/bench64.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --bert --network vgg19 --steps 100 --fp32-steps 0 > $OUT/cfg5.log 2>&1 || exit 1
python tools/bench_brief.py $OUT/bench.log $OUT/bench64.log $OUT/cfg5.log | grep -v "^    [a-z]"
