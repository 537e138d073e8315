"""A/B of ResNet152 layer3's c2 and c3 (14 x 14, 256 -> 256, B = 128): sat_conv3x3_frag (csrc/convblock.hip,
half-image workgroups, weight prefetch 2 / 3 / 4) vs the tile kernel, HIP-event timed back to back."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sat_amd  # noqa: E402
from sat_amd import ops  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) * 1e3 / reps


def main():
    lib = sat_amd._lib.lib()
    dev = torch.device("cuda")
    B = 128
    x = torch.randn(B, 14, 14, 256, device=dev).relu().bfloat16()
    w = (torch.randn(256, 3, 3, 256, device=dev) * 0.03).bfloat16()
    b = torch.randn(256, device=dev) * 0.1
    f = (ops.mfma_frag_layout(w.reshape(256, -1)), b)
    y = torch.empty_like(x)
    flops = 2.0 * B * 196 * 256 * 2304
    us = timeit(lambda: ops.conv2d_nhwc(x, w, b, 1, 1, True, out=y))
    print(f"tile kernel      : {us:7.2f} us  {flops / us / 1e6:7.1f} TFLOP/s  frac {flops / us / 1e6 / 2500:.3f}")
    ref = y.clone()
    for pf in (2, 3, 2 | 16, 2 | 16 | 32, 2 | 64):
        assert lib.sat_conv3x3_frag_set_experiment(pf) == 0
        us = timeit(lambda: ops.conv3x3_frag(x, f, out=y))
        same = torch.equal(y, ref)
        kind = ("slice 2x4 " if pf & 32 else "slice     ") if pf & 16 else ("half-dma  " if pf & 64 else "half-image")
        print(f"{kind} pf {pf & 15}: {us:7.2f} us  {flops / us / 1e6:7.1f} TFLOP/s  frac {flops / us / 1e6 / 2500:.3f}"
              f"  bit-identical {same}")
    lib.sat_conv3x3_frag_set_experiment(2)
    # layer2 c2: 28 x 28, 128 -> 128 (7-row bands)
    x2 = torch.randn(B, 28, 28, 128, device=dev).relu().bfloat16()
    w2 = (torch.randn(128, 3, 3, 128, device=dev) * 0.04).bfloat16()
    b2 = torch.randn(128, device=dev) * 0.1
    f2 = (ops.mfma_frag_layout(w2.reshape(128, -1)), b2)
    y2 = torch.empty_like(x2)
    fl2 = 2.0 * B * 784 * 128 * 1152
    us = timeit(lambda: ops.conv2d_nhwc(x2, w2, b2, 1, 1, True, out=y2))
    print(f"L2c2 tile kernel : {us:7.2f} us  {fl2 / us / 1e6:7.1f} TFLOP/s  frac {fl2 / us / 1e6 / 2500:.3f}")
    ref2 = y2.clone()
    for pf in (2, 3):
        assert lib.sat_conv3x3_frag_set_experiment(pf) == 0
        us = timeit(lambda: ops.conv3x3_frag(x2, f2, out=y2))
        print(f"L2c2 band pf {pf}   : {us:7.2f} us  {fl2 / us / 1e6:7.1f} TFLOP/s  frac {fl2 / us / 1e6 / 2500:.3f}"
              f"  bit-identical {torch.equal(y2, ref2)}")
    lib.sat_conv3x3_frag_set_experiment(2)
    # c1: 1x1 1024 -> 256
    x1 = torch.randn(B, 14, 14, 1024, device=dev).relu().bfloat16()
    w1 = (torch.randn(256, 1, 1, 1024, device=dev) * 0.03).bfloat16()
    b1 = torch.randn(256, device=dev) * 0.1
    f1 = (ops.mfma_frag_layout(w1.reshape(256, -1)), b1)
    y1 = torch.empty(B, 14, 14, 256, device=dev).bfloat16()
    fl1 = 2.0 * B * 196 * 256 * 1024
    us = timeit(lambda: ops.conv2d_nhwc(x1, w1, b1, 1, 0, True, out=y1))
    print(f"c1 tile kernel   : {us:7.2f} us  {fl1 / us / 1e6:7.1f} TFLOP/s  frac {fl1 / us / 1e6 / 2500:.3f}")
    ref1 = y1.clone()
    us = timeit(lambda: ops.conv1x1_frag(x1, f1, out=y1))
    print(f"c1 frag kernel   : {us:7.2f} us  {fl1 / us / 1e6:7.1f} TFLOP/s  frac {fl1 / us / 1e6 / 2500:.3f}"
          f"  bit-identical {torch.equal(y1, ref1)}")
    # c3: 1x1 256 -> 1024 + identity residual
    x3 = torch.randn(B, 14, 14, 256, device=dev).relu().bfloat16()
    r3 = torch.randn(B, 14, 14, 1024, device=dev).relu().bfloat16()
    w3 = (torch.randn(1024, 1, 1, 256, device=dev) * 0.05).bfloat16()
    b3 = torch.randn(1024, device=dev) * 0.1
    f3 = (ops.mfma_frag_layout(w3.reshape(1024, -1)), b3)
    y3 = torch.empty_like(r3)
    byts = 2.0 * (B * 196 * (256 + 2 * 1024) + 1024 * 256)
    us = timeit(lambda: ops.conv2d_nhwc(x3, w3, b3, 1, 0, True, residual=r3, out=y3))
    print(f"c3 stream kernel : {us:7.2f} us  {byts / us / 1e3:7.1f} GB/s  frac {byts / us / 1e3 / 8000:.3f}")
    ref3 = y3.clone()
    for pf in (2, 3):
        assert lib.sat_conv1x1_res_frag_set_experiment(pf) == 0
        us = timeit(lambda: ops.conv1x1_res_frag(x3, f3, r3, out=y3))
        print(f"c3 frag pf {pf}     : {us:7.2f} us  {byts / us / 1e3:7.1f} GB/s  frac {byts / us / 1e3 / 8000:.3f}"
              f"  bit-identical {torch.equal(y3, ref3)}")
    lib.sat_conv1x1_res_frag_set_experiment(2)


if __name__ == "__main__":
    main()
