"""GPU time of sat_images_to_input for a COCO-shaped batch (B x 480x640 uint8 -> 224x224) in each
output layout, with algorithmic bytes (uint8 input read once + output written once) vs 8 TB/s.
    python tools/images_bench.py [B]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import sat_amd  # noqa: E402
from sat_amd import ops, _lib as Lb  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
rng = np.random.default_rng(0)
imgs = [rng.integers(0, 256, (480, 640, 3), dtype=np.uint8) for _ in range(B)]
packed = sat_amd.PackedImages.from_arrays(imgs).to("cuda")
in_bytes = packed.pixels.numel()
res = {}
for name, layout, dt in (("nchw_f32", Lb.IMG_NCHW, torch.float32), ("nhwc8_bf16", Lb.IMG_NHWC, torch.bfloat16),
                         ("s2d16_bf16", Lb.IMG_S2D16, torch.bfloat16)):
    out = ops.images_to_input(packed, layout, dt)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        ops.images_to_input(packed, layout, dt)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    by = in_bytes + out.numel() * out.element_size()
    res[name] = {"us": round(us, 1), "alg_bytes": by, "GBps": round(by / us / 1e3, 1), "frac_8TBps": round(by / us / 8e6, 3)}
print(json.dumps({"B": B, "in": "480x640 uint8", "out": "224x224", "layouts": res}))
