set -u
OUT=gpurun_out/r6_s59; mkdir -p $OUT
i=0
for cfg in NONE=1 HIP_FORCE_DEV_KERNARG=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 NONE=2; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --fp32-steps 0 > $OUT/e${i}_${cfg%%=*}.log 2>&1 || exit $?
  echo "== $cfg"; python tools/bench_brief.py $OUT/e${i}_${cfg%%=*}.log | head -30 || true
done
