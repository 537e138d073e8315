timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "conv or epilogue or encoder or fill" > gpurun_out/t79.log 2>&1; tail -2 gpurun_out/t79.log; grep -n "^E " gpurun_out/t79.log | head -8
SHAPES=L1_c1,L1_c3,L2_c1,L2_c2,L2_c3,L3_c1,L3_c2,L3_c3,L4_c2 CONFIGS="0,0,1" bash tools/ab_conv.sh
