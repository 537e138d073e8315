set -u
OUT=gpurun_out/r3_s7; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_shapes.py tests/test_gpu_dp.py tests/test_gpu_parity.py -k "decoder or attention or shapes or dp or bleu or beam or two_decoder" > $OUT/tests.log 2>&1; rc=$?; tail -5 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
bash tools/r3_stamps.sh
