set -u
OUT=gpurun_out/r3_s20; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; grep -E "^FAILED|Error" $OUT/tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
python tools/bench_brief.py $OUT/bench.log | grep -v "^    [a-z]"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python tools/prof_summary.py $OUT/prof $OUT/prof.log $OUT/prof_summary.json > /dev/null; python -c "
import json; d=json.load(open('$OUT/prof_summary.json')); print(d.get('bench'), d.get('rocprof_dominant'), d.get('trace'))
nl = d.get('decoder_nonloop') or {}; print('nonloop', nl.get('launches'), nl.get('us'))
for r in (nl.get('top') or [])[:12]: print(r)"
