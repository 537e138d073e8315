set -u
OUT=gpurun_out/r3_s13; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention or transposed or decoder_eval or decoder_train" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --batch 64 --steps 100 --no-cpu-baseline --fp32-steps 0 > $OUT/bench64.log 2>&1 || { tail -20 $OUT/bench64.log; exit 1; }
timeout -k 10 300 python bench.py --batch 64 --steps 100 --no-cpu-baseline --fp32-steps 0 --conv-slices 3 > $OUT/bench64_s3.log 2>&1 || { tail -20 $OUT/bench64_s3.log; exit 1; }
python tools/bench_brief.py $OUT/bench64.log $OUT/bench64_s3.log | grep -v "^    L\|^    [a-z]"
timeout -k 10 300 env B=128 CONFIGS="1:0,0,0,0;1:2,0,0,0;1:0,4,0,0;1:2,4,0,0;1:0,2,0,0" python tools/bench_decoder_splits.py > $OUT/splits128.log 2>&1; grep -v amdgpu $OUT/splits128.log
timeout -k 10 200 python tools/conv_class_ab.py 128 > $OUT/conv_ab.log 2>&1; grep -v amdgpu $OUT/conv_ab.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python tools/prof_summary.py $OUT/prof $OUT/prof.log $OUT/prof_summary.json > /dev/null; python -c "
import json; d=json.load(open('$OUT/prof_summary.json')); print(d.get('bench'), d.get('rocprof_dominant'), d.get('trace'))
nl = d.get('decoder_nonloop') or {}; print('nonloop', nl.get('launches'), nl.get('us'))
for r in (nl.get('top') or [])[:30]: print(r)"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-graph --fp32-steps 0 --no-diagnostics > $OUT/pmc_fetch.log 2>&1 || { tail -5 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-graph --fp32-steps 0 --no-diagnostics > $OUT/pmc_write.log 2>&1 || { tail -5 $OUT/pmc_write.log; exit 1; }
python tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write resnet152 128 $OUT/pmc_traffic_resnet152.json | tail -30
find $OUT/pmc_fetch $OUT/pmc_write -name "*.csv" -size +20M -delete
