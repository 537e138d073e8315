"""Time one ResNet152 identity bottleneck as the fused launch (sat_bottleneck_fused, csrc/convblock.hip) against the
three launches the trunk otherwise issues (c1, c2 on the half-image / band kernel, c3 + residual), back to back between
HIP events, outputs compared bit for bit (GPU).

    python tools/block_ab.py [B ...]
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import sat_amd  # noqa: E402,F401
from sat_amd import ops  # noqa: E402

DEV = torch.device("cuda")
# name, H, Cin, Cmid
BLOCKS = [("layer2 block 28x28 512->128", 28, 512, 128), ("layer3 block 14x14 1024->256", 14, 1024, 256)]


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    en.synchronize()
    return st.elapsed_time(en) / reps * 1e3


def main():
    for B in [int(a) for a in sys.argv[1:]] or [128, 64]:
        for name, H, C, M in BLOCKS:
            g = torch.Generator(device=DEV).manual_seed(B + H)
            x = torch.randn(B, H, H, C, device=DEV, generator=g).relu().bfloat16()
            ws = []
            for cout, cin, k in ((M, C, 1), (M, M, 3), (C, M, 1)):
                w = (torch.randn(cout, k, k, cin, device=DEV, generator=g) * math.sqrt(2.0 / (k * k * cin))).bfloat16()
                ws.append((w, 0.1 * torch.randn(cout, device=DEV, generator=g)))
            frags = [(ops.mfma_frag_layout(w.reshape(w.shape[0], -1)), b) for w, b in ws]

            def unfused():
                if ops.conv1x1_frag_supported(H, H, C, M, torch.bfloat16):
                    y1 = ops.conv1x1_frag(x, frags[0])
                else:
                    y1 = ops.conv2d_nhwc(x, ws[0][0], ws[0][1], 1, 0, True)
                y2 = ops.conv3x3_frag(y1, frags[1])
                return ops.conv2d_nhwc(y2, ws[2][0], ws[2][1], 1, 0, True, residual=x)

            def fused():
                return ops.bottleneck_fused(x, *frags)
            same = torch.equal(unfused(), fused())
            tu, tf = timed(unfused), timed(fused)
            flops = 2.0 * B * H * H * (C * M + 9 * M * M + M * C)
            print(f"B {B:4d} {name:30s} three launches {tu:7.1f} us   fused {tf:7.1f} us ({flops / tf / 1e6:6.0f} TF/s)"
                  f"   x{tu / tf:.2f}  {'bit-identical' if same else 'DIFFERENT'}", flush=True)


if __name__ == "__main__":
    main()
