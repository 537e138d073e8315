"""Time the decoder's batched (non-per-step) GEMMs at the bench shape one by one (GPU).

B = 128, T = 27 (R = B * 26 = 3328 rows), V = 10000, E = 512, D = 2048, L = 49, bf16 operands: the hoisted
Ws = a W^T, the input / output head products of the forward, and the weight / input gradients of the backward
(decoder.hip).  Each product is re-issued back to back between HIP events: the library default (the split-K kernel,
gemmsplit.hip, for the fp32-output products with a k-major operand), the 128x128 tile kernel (SatPolicy.split_gemm
= 1) and, with --forms, each split-K form (tile height x split count).

    python tools/head_gemms.py [--forms] [--reps 10] [--torch]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import sat_amd  # noqa: E402
from sat_amd import ops  # noqa: E402

B, T, V, E, D, L = 128, 27, 10000, 512, 2048, 49
R = B * (T - 1)
HG = 5 * E + D
DEV = torch.device("cuda")

RELU = sat_amd._lib.ACT_RELU
# name, M, N, K, transA, transB, c dtype, beta[, act]
SHAPES = [
    ("Ws = a.W^T (fwd)", B * L, E, D, False, False, torch.bfloat16, 0.0),
    ("x gates = emb.W_ih[:, :E]^T", R, 4 * E, E, False, False, torch.float32, 0.0),
    ("f_z (fwd, ReLU)", R, E, D, False, False, torch.float32, 0.0, RELU),
    ("f_out logits (fwd, ReLU)", R, V, E, False, False, torch.bfloat16, 0.0, RELU),
    ("dW f_out", V, E, R, True, True, torch.float32, 0.0),
    ("dX f_out", R, E, V, False, True, torch.float32, 0.0),
    ("dW f_z", E, D, R, True, True, torch.float32, 0.0),
    ("dX f_z", R, D, E, False, True, torch.float32, 0.0),
    ("dW attention.W", E, D, B * L, True, True, torch.float32, 0.0),
    ("dW [U; f_beta; W_hh]", HG, E, R, True, True, torch.float32, 0.0),
    ("dW W_ih[:, :E]", 4 * E, E, R, True, True, torch.float32, 0.0),
    ("dW W_ih[:, E:]", 4 * E, D, R, True, True, torch.float32, 0.0),
    ("dX embedding", R, E, 4 * E, False, True, torch.float32, 0.0),
]
# (label, split_gemm, split_k)
FORMS = [("128x1", 2, 1), ("128x2", 2, 2), ("128x3", 2, 3), ("128x4", 2, 4), ("128x6", 2, 6), ("128x8", 2, 8),
         ("256x1", 3, 1), ("256x2", 3, 2), ("256x3", 3, 3), ("256x4", 3, 4)]


def operands(M, N, K, ta, tb, cdt):
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    A = (torch.randn(K, M, device=DEV, generator=g) if ta else torch.randn(M, K, device=DEV, generator=g)).bfloat16()
    Bm = (torch.randn(K, N, device=DEV, generator=g) if tb else torch.randn(N, K, device=DEV, generator=g)).bfloat16()
    C = torch.empty(M, N, device=DEV, dtype=cdt)
    return A, Bm, C


def time_one(A, Bm, C, ta, tb, beta, policy, reps, act=0):
    def go():
        ops.gemm(A, Bm, C, transA=ta, transB=tb, beta=beta, act=act, policy=policy)
    for _ in range(2):
        go()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        go()
    en.record()
    en.synchronize()
    return st.elapsed_time(en) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--forms", action="store_true", help="every split-K form (tile height x splits) of the k-major products")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--torch", action="store_true",
                    help="calibration: torch.matmul (hipBLASLt) of the same bf16 operands, bf16 output")
    a = ap.parse_args()
    tot_us = tot_f = tot_tile = tot_lib = 0.0
    for name, M, N, K, ta, tb, cdt, beta, *rest in SHAPES:
        act = rest[0] if rest else 0
        A, Bm, C = operands(M, N, K, ta, tb, cdt)
        f = 2.0 * M * N * K
        us = time_one(A, Bm, C, ta, tb, beta, None, a.reps, act)
        tot_us += us
        tot_f += f
        us_tile = time_one(A, Bm, C, ta, tb, beta, sat_amd.Policy(split_gemm=1), a.reps, act)
        tot_tile += us_tile
        line = f"{name:30s} M {M:5d} N {N:5d} K {K:5d} {'T' if ta else 'N'}{'T' if tb else 'N'}  {us:8.1f} us " \
               f"{f / us / 1e6:7.1f} TF/s  [tile kernel {us_tile:.1f} us]"
        if a.forms and (ta or tb) and cdt == torch.float32:
            alt = []
            for label, sg, sk in FORMS:
                try:
                    alt.append(f"{label}:{time_one(A, Bm, C, ta, tb, beta, sat_amd.Policy(split_gemm=sg, split_k=sk), a.reps, act):.1f}")
                except RuntimeError:
                    alt.append(f"{label}:-")
            line += "  [" + " ".join(alt) + "]"
        if a.torch:
            At = A.t() if ta else A          # [M, K] view
            Bt = Bm if tb else Bm.t()        # [K, N] view
            out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)

            def mm():
                torch.matmul(At, Bt, out=out)
            for _ in range(2):
                mm()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(a.reps):
                mm()
            en.record()
            en.synchronize()
            us_lib = st.elapsed_time(en) / a.reps * 1e3
            tot_lib += us_lib
            line += f"  [calibration, torch.matmul / hipBLASLt bf16 out: {us_lib:.1f} us]"
        print(line, flush=True)
    print(f"total {tot_us:.1f} us for {tot_f / 1e9:.1f} GFLOP = {tot_f / tot_us / 1e6:.1f} TF/s "
          f"(tile kernel for the k-major products: {tot_tile:.1f} us"
          + (f"; torch.matmul calibration {tot_lib:.1f} us" if a.torch else "") + ")", flush=True)


if __name__ == "__main__":
    main()
