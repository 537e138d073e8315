timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "tile_configs or fast_conv" > gpurun_out/t89.log 2>&1; tail -1 gpurun_out/t89.log; grep -n "^E " gpurun_out/t89.log | head -5
SHAPES=L2_c1,L2_c2,L3_c1,L3_c2,L3_c3,L4_c2 CONFIGS="0,0,1;0,3,1" bash tools/ab_conv.sh
