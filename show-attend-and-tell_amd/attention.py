"""Attention module (reference: attention.py:5-21).

Same constructor, submodules (``U``, ``W``, ``v``) and state_dict keys as the
reference; ``forward(img_features, hidden_state) -> (context, alpha)`` runs the
fused HIP attention kernel (scores, softmax over L, annotation-weighted context)
after two MFMA GEMMs for ``U h`` and ``W a``.

Inside the decoder the attention step is not called through this module: the
decoder's fused time loop (sat_decoder_forward) runs the same kernel with the
loop-invariant ``W a`` hoisted out of the loop.  This standalone forward is
inference-only (no autograd graph), like the reference's use in
``Decoder.caption`` (decoder.py:160-269).
"""
import torch
import torch.nn as nn

from . import _lib as L


class Attention(nn.Module):
    def __init__(self, encoder_dim, embedding_size):
        super().__init__()
        self.U = nn.Linear(embedding_size, embedding_size)
        self.W = nn.Linear(encoder_dim, embedding_size)
        self.v = nn.Linear(embedding_size, 1)
        self.tanh = nn.Tanh()
        self.softmax = nn.Softmax(1)

    def forward(self, img_features, hidden_state):
        L.require_device(img_features, hidden_state, self.U.weight)
        B, Lh, D = img_features.shape
        E = self.U.weight.shape[0]
        dt = L.dtype_code(img_features.dtype)
        feats = img_features.contiguous()
        h = hidden_state.contiguous().float()
        dev = feats.device
        w_lp = None
        if dt == L.SAT_BF16:
            from .ops import cast_
            w_lp = cast_(self.W.weight.detach().contiguous(), torch.empty(E, D, device=dev, dtype=torch.bfloat16))
        scratch = torch.empty(B * Lh * E + B * E, device=dev, dtype=torch.float32)
        context = torch.empty(B, D, device=dev, dtype=torch.float32)
        alpha = torch.empty(B, Lh, device=dev, dtype=torch.float32)
        p = lambda t: L.ptr(t.detach().contiguous())  # noqa: E731
        L.check(L.lib().sat_attention_forward(B, Lh, D, E, dt, L.ptr(feats), L.ptr(h), p(self.U.weight), p(self.U.bias),
                                              p(self.W.weight), L.ptr(w_lp), p(self.W.bias), p(self.v.weight),
                                              p(self.v.bias), L.ptr(scratch), L.ptr(context), L.ptr(alpha),
                                              L.stream_of(context)), "sat_attention_forward")
        return context, alpha
