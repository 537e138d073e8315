set -e
mkdir -p gpurun_out/r5_s7
for i in 1 2; do
  timeout -k 10 200 python tools/head_gemms.py > gpurun_out/r5_s7/hg_prod_$i.log 2>&1
  SAT_HIP_LIB_TUNING=show-attend-and-tell_amd/libsat_hip_norel.so timeout -k 10 200 python tools/head_gemms.py > gpurun_out/r5_s7/hg_norel_$i.log 2>&1
done
grep -h total gpurun_out/r5_s7/hg_*.log
bash tools/session.sh r5_s7 ab:prod abl:norel:norel ab:prod abl:norel:norel
