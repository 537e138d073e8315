"""Measurement helpers for bench.py (not part of the training path).

decoder_step_kernels(): the per-time-step decoder kernels (the fused attention + LSTM step of
SURVEY.md 8(d), plus the skinny per-step GEMMs) timed live with HIP events: one C-ABI forward and
backward fill a private workspace, then sat_decoder_step_bench re-issues each kernel group of the
middle time step back to back.  Returned with each group's algorithmic HBM bytes (inputs read
once, outputs written once) so bench.py can report achieved GB/s against 8 TB/s.

decoder_flops(): algorithmic FLOPs of one decoder train step per image (forward with W.a hoisted,
backward = 2x forward), the decoder part of SURVEY.md 8(d)'s whole-step roofline.
"""
import ctypes

import torch

from . import _lib as L

GROUPS = ("h_gemm", "attn_fwd", "ctx_gemm", "lstm_fwd", "lstm_bwd", "dgated_gemm", "attn_bwd", "dh_gemm")
# the fused attention + LSTM step kernels (the HBM-bound part of SURVEY 8(d))
FUSED = ("attn_fwd", "lstm_fwd", "lstm_bwd", "attn_bwd")


def decoder_flops(L_, D, E, V, T, ado=True, attention=True):
    """FLOPs per image of decoder forward + backward (reference decoder.py:69-158 with Ws hoisted)."""
    T1 = T - 1
    fwd = 2 * 2 * D * E                                   # init_h, init_c
    if attention:
        fwd += 2 * L_ * D * E                             # Ws = a W^T (once, hoisted)
    step = 2 * 4 * E * (E + D) + 2 * 4 * E * E            # LSTM W_ih, W_hh
    if attention:
        step += 2 * E * E + 2 * E * D                     # U h, f_beta h
        step += 2 * L_ * E + 2 * L_ * D                   # scores (v . tanh), context
    step += (2 * E * E + 2 * D * E + 2 * E * V) if ado else 2 * E * V
    fwd += T1 * step
    return 3.0 * fwd


def step_group_bytes(B, L_, D, E, T, ts, attention=True, ado=True):
    """Algorithmic HBM bytes of one launch group per time step (see GROUPS)."""
    HG = 5 * E + D if attention else 4 * E
    NS = -(-D // (64 * (8 if ts == 2 else 4)))
    by = {
        "h_gemm": HG * E * ts + B * E * ts + B * HG * 4,
        "attn_fwd": B * L_ * E * ts + B * L_ * D * ts + B * (E + D) * 4 + E * 4
                    + B * L_ * 4 + B * D * (4 + ts + 4 + ts) + B * E * 4,
        "ctx_gemm": 4 * E * D * ts + B * D * ts + B * 4 * E * 4,
        "lstm_fwd": 3 * B * 4 * E * 4 + B * E * 4 + B * 4 * E * 4 + 3 * B * E * 4 + B * E * ts,
        "lstm_bwd": B * 4 * E * 4 + 4 * B * E * 4 + B * E + 2 * B * E * 4 + B * 4 * E * (4 + ts),
        "dgated_gemm": 4 * E * D * ts + B * 4 * E * ts + B * D * 4,
        "attn_bwd": (B * L_ * D * ts + B * D * 4 * (4 if ado else 3) + B * D * (4 + ts) + B * NS * L_ * 4)
                    + (B * L_ * E * ts + B * E * 4 + 2 * B * L_ * 4 + B * NS * L_ * 4 + B * E * (4 + ts)
                       + 2 * B * E * 4 + B * L_ * 4),
        "dh_gemm": HG * E * ts + B * HG * ts + B * E * 4,
    }
    if not attention:
        for k in ("attn_fwd", "ctx_gemm", "dgated_gemm", "attn_bwd"):
            by[k] = 0
    return by


def decoder_step_kernels(dec, feats, captions, reps=20):
    """{group: avg us per launch} for the decoder's per-step kernel groups at step (T-1)/2 (the
    module's current train/eval mode and dtype), plus per-group algorithmic bytes."""
    from .decoder import _DecoderFn  # noqa: F401  (same argument setup as the autograd function)
    lib = L.lib()
    dec._ensure_flat(feats.device)
    if feats.dtype == torch.bfloat16:
        dec._ensure_lp()
    dims = dec._dims(feats, captions)
    lay = dec._layout()
    ws_bytes = lib.sat_decoder_workspace_bytes(ctypes.byref(dims))
    dev = feats.device
    ws = torch.empty(ws_bytes, device=dev, dtype=torch.uint8)
    B, T1 = dims.B, dims.T - 1
    preds = torch.empty(B, T1, dims.V, device=dev, dtype=feats.dtype)
    alphas = torch.empty(B, T1, dims.L, device=dev, dtype=torch.float32)
    tokens = torch.empty(B, T1, device=dev, dtype=torch.int32)
    lp = dec._flat_lp if dims.dtype == L.SAT_BF16 else None
    stream = L.stream_of(preds)
    caps = captions.contiguous().long()
    L.check(lib.sat_decoder_forward(ctypes.byref(dims), ctypes.byref(lay), L.ptr(dec._flat), L.ptr(lp), L.ptr(feats),
                                    L.ptr(caps), None, L.ptr(ws), ws_bytes, L.ptr(preds), L.ptr(alphas),
                                    L.ptr(tokens), stream), "sat_decoder_forward")
    d_preds = torch.randn_like(preds, dtype=torch.float32).to(preds.dtype) * 1e-3
    d_alphas = torch.randn_like(alphas) * 1e-3
    grads = torch.zeros_like(dec._flat)
    for phase in (1, 2):
        L.check(lib.sat_decoder_backward(ctypes.byref(dims), ctypes.byref(lay), L.ptr(dec._flat), L.ptr(lp),
                                         L.ptr(feats), L.ptr(ws), ws_bytes, L.ptr(preds), L.ptr(alphas),
                                         L.ptr(d_preds), L.ptr(d_alphas), L.ptr(grads), 0, phase, stream),
                "sat_decoder_backward")
    us = (ctypes.c_float * 8)()
    L.check(lib.sat_decoder_step_bench(ctypes.byref(dims), ctypes.byref(lay), L.ptr(dec._flat), L.ptr(lp),
                                       L.ptr(feats), L.ptr(ws), ws_bytes, L.ptr(alphas), L.ptr(d_alphas), int(reps),
                                       us, stream), "sat_decoder_step_bench")
    times = {g: float(us[i]) for i, g in enumerate(GROUPS)}
    ts = 2 if feats.dtype == torch.bfloat16 else 4
    by = step_group_bytes(B, dims.L, dims.D, dims.E, dims.T, ts, bool(dims.attention), bool(dims.ado))
    return times, by
