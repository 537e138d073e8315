# A/B of CU-partitioned decoder / encoder streams (bench.py --cu-split)
set -u
OUT=gpurun_out/${1:-s42}; mkdir -p $OUT
run() { local tag=$1; shift
  timeout -k 10 200 python bench.py --steps 60 --no-cpu-baseline --fp32-steps 0 --no-diagnostics "$@" > $OUT/$tag.log 2>&1 || { echo "$tag FAILED"; tail -5 $OUT/$tag.log; exit 1; }
  echo "$tag $* $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.log) $(grep -o '"graph_ms_per_step": [0-9.]*' $OUT/$tag.log)"; }
run base --bwd split --enc-split none
run base_l3 --bwd split
for n in 32 64 96; do for lay in strided contig; do
  run cu${n}${lay} --bwd split --enc-split none --cu-split $n --cu-layout $lay
done; done
run cu64s_t32 --bwd split --enc-split none --cu-split 64 --split-target 32
run cu64s_t128 --bwd split --enc-split none --cu-split 64 --split-target 128
