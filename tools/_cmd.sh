SHAPES=L1_c3,L2_c1,L2_c3,L3_c1,L3_c3,L3_c2 CONFIGS="0,0,1;3,2,1;2,2,1" timeout -k 10 300 python tools/bench_conv.py 2>&1 | grep -v amdgpu.ids
