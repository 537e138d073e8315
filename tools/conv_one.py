"""Run one conv shape of the ResNet152 trunk repeatedly (for rocprofv3 counter passes).

    python tools/conv_one.py L3_c3 [reps] [tile] [stages]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import sat_amd  # noqa: E402
from sat_amd import ops  # noqa: E402

SHAPES = {"L1_c3": (56, 64, 256, 1, 1, 0, 1), "L2_c3": (28, 128, 512, 1, 1, 0, 1), "L3_c1": (14, 1024, 256, 1, 1, 0, 0),
          "L3_c2": (14, 256, 256, 3, 1, 1, 0), "L3_c3": (14, 256, 1024, 1, 1, 0, 1), "L2_c2": (28, 128, 128, 3, 1, 1, 0),
          "stem": (224, 8, 64, 7, 2, 3, 0),
          "L3_c2_16": (16, 256, 256, 3, 1, 1, 0), "L3_c1_16": (16, 1024, 256, 1, 1, 0, 0)}
name = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
tile = int(sys.argv[3]) if len(sys.argv) > 3 else 0
stages = int(sys.argv[4]) if len(sys.argv) > 4 else 0
H, C, Co, k, s, p, r = SHAPES[name]
B = 128
x = torch.randn(B, H, H, C, device="cuda").bfloat16()
w = (torch.randn(Co, k, k, C, device="cuda") / (k * k * C) ** 0.5).bfloat16()
b = torch.randn(Co, device="cuda")
OH = (H + 2 * p - k) // s + 1
res = torch.randn(B, OH, OH, Co, device="cuda").bfloat16() if r else None
y = torch.empty(B, OH, OH, Co, device="cuda", dtype=torch.bfloat16)
sat_amd._lib.lib().sat_fast_gemm_set_config(stages, tile, 1)
for _ in range(reps):
    ops.conv2d_nhwc(x, w, b, s, p, True, residual=res, out=y)
torch.cuda.synchronize()
print("done", name, reps)
