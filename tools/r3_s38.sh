set -u
OUT=gpurun_out/r3_s38; mkdir -p $OUT; export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_$C -o run --output-format csv -- \
    python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-graph --fp32-steps 0 --no-diagnostics > $OUT/pmc_$C.log 2>&1
  rc=$?; echo "$C rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc_$C.log; exit $rc; }
done
python tools/pmc_traffic.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE resnet152 128 $OUT/pmc_traffic_resnet152.json > $OUT/pmc_summary.log 2>&1 || { tail -5 $OUT/pmc_summary.log; exit 1; }
python -c "
import json; d=json.load(open('$OUT/pmc_traffic_resnet152.json'))
for k,v in d['classes'].items(): print(k, v['ratio_to_algorithmic'], round(v['hbm_bytes_per_launch']/1e6,1))
print(d['unit_check_input_layout'])"
find $OUT -name "*counter_collection.csv" -size +20M -delete
