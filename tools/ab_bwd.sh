set -u
mkdir -p gpurun_out/s41
for v in side serial split; do
  for ov in "" "--no-overlap"; do
    timeout -k 10 200 python bench.py --steps 60 --no-cpu-baseline --fp32-steps 0 --no-diagnostics --bwd $v $ov > gpurun_out/s41/$v$ov.log 2>&1 || exit $?
    echo "$v $ov $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s41/$v$ov.log)"
  done
done
