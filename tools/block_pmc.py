"""Runs only the fused bottleneck kernel (B = 128, 10 launches) for rocprofv3 PMC passes:
    rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d DIR -o run --output-format csv -- python tools/block_pmc.py [abl]"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import sat_amd  # noqa: E402
from sat_amd import ops  # noqa: E402

abl = int(sys.argv[1]) if len(sys.argv) > 1 else 0
B, dev = 128, "cuda"
g = torch.Generator().manual_seed(0)
x = torch.randn(B, 14, 14, 1024, generator=g).relu().bfloat16().to(dev)
frags = []
for cout, cin, k in ((256, 1024, 1), (256, 256, 3), (1024, 256, 1)):
    w = (torch.randn(cout, k * k * cin, generator=g) * math.sqrt(2.0 / (k * k * cin))).bfloat16().to(dev)
    frags.append((ops.mfma_frag_layout(w), (0.1 * torch.randn(cout, generator=g)).to(dev)))
assert sat_amd._lib.lib().sat_bottleneck_set_experiment(2, abl) == 0
y = torch.empty_like(x)
for _ in range(10):
    ops.bottleneck_fused(x, *frags, out=y)
torch.cuda.synchronize()
print("done")
