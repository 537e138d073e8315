set -u
OUT=gpurun_out/r3_s41; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-tf --no-cpu-baseline --fp32-steps 0 > $OUT/cfg4.log 2>&1 || { tail -5 $OUT/cfg4.log; exit 1; }
python tools/bench_brief.py $OUT/cfg4.log | head -2
timeout -k 10 300 python bench.py --bert --network vgg19 --fp32-steps 0 > $OUT/cfg5.log 2>&1 || { tail -5 $OUT/cfg5.log; exit 1; }
python tools/bench_brief.py $OUT/cfg5.log | head -2
