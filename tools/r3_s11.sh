set -u
OUT=gpurun_out/r3_s11; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "skinny or transposed or attention_backward or decoder_split" > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 env B=128 python tools/bench_decoder_splits.py > $OUT/splits128.log 2>&1; grep -v amdgpu $OUT/splits128.log
timeout -k 10 300 env B=64 python tools/bench_decoder_splits.py > $OUT/splits64.log 2>&1; grep -v amdgpu $OUT/splits64.log
