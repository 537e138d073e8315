"""A/B of the 64 -> 64 3x3 convs: conv3x3_ws_kernel (csrc/conv3x3ws.hip) vs the implicit-GEMM tile kernel,
HIP-event timed back to back (B = 128: ResNet152 layer1 c2 at 56 x 56, VGG19 conv1_2 at 224 x 224)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sat_amd  # noqa: E402
from sat_amd import ops  # noqa: E402


def main():
    lib = sat_amd._lib.lib()
    dev = torch.device("cuda")
    for name, H, C, KK, pad in (("L1c2", 56, 64, 3, 1), ("vgg_conv1_2", 224, 64, 3, 1), ("stem_s2d", 112, 16, 4, 2)):
        x = torch.randn(128, H, H, C, device=dev).bfloat16()
        w = (torch.randn(64, KK, KK, C, device=dev) * 0.05).bfloat16()
        b = torch.randn(64, device=dev)
        y = torch.empty(128, H, H, 64, device=dev).bfloat16()
        for mode in ((1, 0, 1, 0) + tuple(1 | (b << 1) for b in (2, 4, 6)) if len(sys.argv) > 1 else (1, 0, 1, 0)):
            assert lib.sat_conv3x3_ws_set_mode(mode) == 0
            for _ in range(3):
                ops.conv2d_nhwc(x, w, b, 1, pad, True, out=y, out_hw=(H, H))
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            st.record()
            for _ in range(reps):
                ops.conv2d_nhwc(x, w, b, 1, pad, True, out=y, out_hw=(H, H))
            en.record()
            torch.cuda.synchronize()
            us = st.elapsed_time(en) * 1e3 / reps
            flops = 2 * 128 * H * H * 64 * KK * KK * C
            byts = 2 * 128 * H * H * (64 + C)
            print(f"{name:12s} mode {mode:2d}: {us:8.1f} us  {flops / us / 1e6:7.1f} TFLOP/s  {byts / us / 1e3:7.1f} GB/s")
    lib.sat_conv3x3_ws_set_mode(1)


if __name__ == "__main__":
    main()
