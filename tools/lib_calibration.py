"""Calibration only (not product code): time the vendor libraries on the ResNet152 conv shapes
(B=128, bf16) -- MIOpen conv2d (channels_last) and hipBLASLt GEMM of the same M x N x K -- next to
this build's LDS-DMA conv kernel, in one process with interleaved rounds.

    python tools/lib_calibration.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
import sat_amd  # noqa: E402
from sat_amd import ops  # noqa: E402

B = 128
SHAPES = [("L1_c2", 56, 64, 64, 3, 1, 1, 0), ("L1_c3", 56, 64, 256, 1, 1, 0, 1), ("L2_c2", 28, 128, 128, 3, 1, 1, 0),
          ("L2_c3", 28, 128, 512, 1, 1, 0, 1), ("L3_c1", 14, 1024, 256, 1, 1, 0, 0), ("L3_c2", 14, 256, 256, 3, 1, 1, 0),
          ("L3_c3", 14, 256, 1024, 1, 1, 0, 1), ("L4_c2", 7, 512, 512, 3, 1, 1, 0)]


def timeit(fn, reps=10):
    fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    en.synchronize()
    return st.elapsed_time(en) / reps * 1e3


for name, H, C, Co, k, s, p, r in SHAPES:
    OH = (H + 2 * p - k) // s + 1
    M, N, K = B * OH * OH, Co, k * k * C
    x = torch.randn(B, H, H, C, device="cuda").bfloat16()
    w = (torch.randn(Co, k, k, C, device="cuda") / (k * k * C) ** 0.5).bfloat16()
    bias = torch.randn(Co, device="cuda")
    res = torch.randn(B, OH, OH, Co, device="cuda").bfloat16() if r else None
    y = torch.empty(B, OH, OH, Co, device="cuda", dtype=torch.bfloat16)
    xc = x.permute(0, 3, 1, 2)                      # NCHW view of NHWC memory = channels_last
    wc = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
    bb = bias.bfloat16()
    A = torch.randn(M, K, device="cuda").bfloat16()
    Bm = torch.randn(N, K, device="cuda").bfloat16()
    arms = {
        "sat": lambda: ops.conv2d_nhwc(x, w, bias, s, p, True, residual=res, out=y),
        "miopen": lambda: F.conv2d(xc, wc, bb, s, p),
        "blaslt": lambda: torch.mm(A, Bm.t()),
    }
    t = {a: [] for a in arms}
    for _ in range(5):
        for a, fn in arms.items():
            t[a].append(timeit(fn))
    fl = 2.0 * M * N * (3 * k * k if C == 8 else K)
    line = f"{name:6s} {M}x{N}x{K}"
    for a in arms:
        us = statistics.median(t[a])
        line += f"  {a}: {us:7.1f}us {fl / us / 1e6:6.0f}TF"
    print(line, flush=True)
