set -u
OUT=gpurun_out/r3_s14; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention or transposed or decoder or production or skinny" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 env B=128 python tools/bench_decoder_splits.py > $OUT/splits128.log 2>&1; grep -v amdgpu $OUT/splits128.log
timeout -k 10 300 env B=64 python tools/bench_decoder_splits.py > $OUT/splits64.log 2>&1; grep -v amdgpu $OUT/splits64.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "frag" > $OUT/tests_frag.log 2>&1; rc=$?; tail -2 $OUT/tests_frag.log; [ $rc -eq 0 ] || exit $rc
for m in 2 4 5; do timeout -k 10 300 python bench.py --batch 64 --steps 100 --no-cpu-baseline --fp32-steps 0 --conv-slices $m > $OUT/bench64_s$m.log 2>&1 || exit 1; done
python tools/bench_brief.py $OUT/bench64_s2.log $OUT/bench64_s4.log $OUT/bench64_s5.log | grep -v "^    [a-zL]"
timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --fp32-steps 0 > $OUT/bench.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --fp32-steps 0 --enc-start phase2 > $OUT/bench_ph2.log 2>&1 || exit 1
python tools/bench_brief.py $OUT/bench.log $OUT/bench_ph2.log | grep -v "^    [a-zL]"
timeout -k 10 300 python tools/head_gemms.py --split > $OUT/head_gemms.log 2>&1; grep -v amdgpu $OUT/head_gemms.log
