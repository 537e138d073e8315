# tools/debug_policy_edit2.py against diagnostics builds (one per reverted source)
mkdir -p gpurun_out/$1
shift_tag=$1; shift
for v in "$@"; do
  if [ $v = prod ]; then lib=""; else lib=show-attend-and-tell_amd/libsat_hip_$v.so; fi
  SAT_HIP_LIB_TUNING=$lib timeout -k 10 200 python tools/debug_policy_edit2.py > gpurun_out/$shift_tag/$v.log 2>&1 || exit $?
  echo "== $v"; grep splits2 gpurun_out/$shift_tag/$v.log | cut -c1-400
done
