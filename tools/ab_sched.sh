# A/B of overlapped-step schedules (bench.py knobs); one line per variant: ms/step, encoder graph ms
set -u
OUT=gpurun_out/${1:-sched}; shift; mkdir -p $OUT
i=0
while [ $# -gt 0 ]; do
  i=$((i+1)); args=$1; shift
  timeout -k 10 200 python bench.py --steps 60 --no-cpu-baseline --fp32-steps 0 --no-diagnostics $args > $OUT/v$i.log 2>&1 || { echo "v$i [$args] FAILED"; tail -5 $OUT/v$i.log; exit 1; }
  echo "v$i [$args] $(grep -o '"ms_per_step": [0-9.]*' $OUT/v$i.log) $(grep -o '"graph_ms_per_step": [0-9.]*' $OUT/v$i.log)"
done
