"""Fused caption loss + in-loop metrics (reference: train.py:135-162, utils.py:44-80,101-107).

``caption_loss(preds, alphas, captions, alpha_c, pad_id, skip_ids)`` returns
``(loss, metrics)``: ``loss`` is the reference objective

    CE(pack_padded_sequence(preds, T-2), pack_padded_sequence(captions[:,1:], T-2))
      + alpha_c * ((1 - alphas.sum(1)) ** 2).mean()

and ``metrics`` is a device tensor [CE, att_reg, n_top1, n_top5, n_nonpad,
caption_length] so the train loop can report the reference's meters without
the four per-step host syncs the reference pays.  Both come from one
pass over the logits on the GPU; the backward recomputes softmax from the saved
log-sum-exp (no [B,T-1,V] probability tensor is kept).
"""
import torch

from . import _lib as L

PLAIN_PAD, PLAIN_START, PLAIN_EOS = 3, 0, 1          # generate_json_data.py:45-48
BERT_PAD, BERT_CLS, BERT_SEP = 0, 101, 102


class _CaptionLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, preds, alphas, captions, alpha_c, pad_id, skip):
        L.require_device(preds, alphas, captions)
        # no zero-filled gradient for the metrics output (non-differentiable): one fill launch less per backward
        ctx.set_materialize_grads(False)
        B, T1, V = preds.shape
        T = captions.shape[1]
        if T1 != T - 1 or alphas.shape[:2] != (B, T1):
            raise ValueError("caption_loss: preds [B,T-1,V], alphas [B,T-1,L], captions [B,T] expected")
        Lf = alphas.shape[2]
        lib = L.lib()
        ws = torch.empty(lib.sat_caption_loss_workspace_bytes(B, T, Lf), device=preds.device, dtype=torch.uint8)
        out = torch.empty(8, device=preds.device, dtype=torch.float32)
        # the loss in its own 4-byte tensor (a caller may scale it in place: gradient accumulation, loss.mul_ -- a
        # view of a custom Function's output buffer would make autograd reject that), written by the kernel itself
        loss = torch.empty((), device=preds.device, dtype=torch.float32)
        preds_c, alphas_c, caps = preds.contiguous(), alphas.contiguous().float(), captions.contiguous().long()
        L.check(lib.sat_caption_loss_forward_loss_out(B, T, V, Lf, L.dtype_code(preds.dtype), L.ptr(preds_c),
                                                      L.ptr(alphas_c), L.ptr(caps), float(alpha_c), int(pad_id),
                                                      int(skip[0]), int(skip[1]), int(skip[2]), L.ptr(ws), L.ptr(out),
                                                      L.ptr(loss), L.stream_of(out)),
                "sat_caption_loss_forward")
        ctx.save_for_backward(preds_c, caps)
        ctx.ws, ctx.dims, ctx.alpha_c = ws, (B, T, V, Lf), float(alpha_c)
        ctx.relu = bool(getattr(preds, "_sat_relu_logits", False))   # set by sat_amd.Decoder (ado)
        # metrics: a view of the kernel's output (never modified by callers)
        metrics = out[1:7]
        ctx.mark_non_differentiable(metrics)
        return loss, metrics

    @staticmethod
    def backward(ctx, g_loss, g_metrics):
        preds, caps = ctx.saved_tensors
        B, T, V, Lf = ctx.dims
        # bf16 logits whose rows are not 16-B multiples: the gradient goes into rows zero-padded to a multiple of 8,
        # the layout the decoder head's backward GEMMs read (sat_decoder_backward phase bit 8), and is handed on as
        # the [..., :V] view, tagged -- any other consumer sees an ordinary strided tensor
        ld = (V + 7) // 8 * 8 if preds.dtype == torch.bfloat16 and V % 8 else V
        if ld != V:
            d_pad = torch.empty(B, T - 1, ld, device=preds.device, dtype=preds.dtype)
            d_preds = d_pad[..., :V]
        else:
            d_pad = d_preds = torch.empty_like(preds)
        d_alphas = torch.empty(B, T - 1, Lf, device=preds.device, dtype=torch.float32)
        g = (g_loss if g_loss is not None else torch.ones((), device=preds.device)).float().contiguous()
        # with ReLU'd logits the mask of that ReLU is applied here, and the gradient says so
        L.check(L.lib().sat_caption_loss_backward_ld(B, T, V, Lf, L.dtype_code(preds.dtype), L.ptr(preds),
                                                     L.ptr(caps), ctx.alpha_c, L.ptr(ctx.ws), L.ptr(g),
                                                     L.ptr(d_pad), ld, L.ptr(d_alphas), int(ctx.relu),
                                                     L.stream_of(d_preds)),
                "sat_caption_loss_backward")
        if ctx.relu:
            d_preds._sat_relu_masked = True
        if ld != V:
            d_preds._sat_padded_ld = ld
        ctx.ws = None
        return d_preds, d_alphas, None, None, None, None


def caption_loss(preds, alphas, captions, alpha_c=1.0, pad_id=PLAIN_PAD, skip_ids=(PLAIN_PAD, PLAIN_START, PLAIN_EOS)):
    return _CaptionLossFn.apply(preds, alphas, captions, alpha_c, pad_id, tuple(skip_ids))


def special_ids(bert):
    """(pad_id, skip_ids) as train.py:143,174-177 pick them."""
    if bert:
        return BERT_PAD, (BERT_PAD, BERT_CLS, BERT_SEP)
    return PLAIN_PAD, (PLAIN_PAD, PLAIN_START, PLAIN_EOS)


class StepMetrics:
    """Host view of the metrics tensor: one D2H copy when read (not per step)."""

    def __init__(self, loss, metrics):
        self.loss, self.metrics = loss, metrics

    def values(self):
        m = self.metrics.detach().cpu().tolist()
        ce, reg, c1, c5, nonpad, cap_len = m
        acc1 = c1 * 100.0 / nonpad if nonpad > 0 else 0
        acc5 = c5 * 100.0 / nonpad if nonpad > 0 else 0
        return dict(loss=float(self.loss.detach().cpu()), ce=ce, att_reg=reg, acc1=acc1, acc5=acc5,
                    caption_length=int(cap_len))


class RunningMeters:
    """The reference's three AverageMeters (utils.py:4-19; train.py:179-181: loss, top-1, top-5, each
    weighted by the step's caption length) accumulated ON THE DEVICE every step: update() issues
    four tiny elementwise ops and never synchronises; read() is the one host copy per log line."""

    def __init__(self, device):
        self.acc = torch.zeros(4, device=device, dtype=torch.float64)   # sum loss*n, acc1*n, acc5*n, n
        self.last = None

    def update(self, loss, metrics):
        # metrics = [CE, att_reg, n_top1, n_top5, n_nonpad, caption_length] (float32 device tensor)
        m = metrics.detach().double()
        n = m[5]
        nonpad = m[4].clamp_min(1.0)
        has = (m[4] > 0).double()
        step = torch.stack([loss.detach().double() * n, m[2] * 100.0 / nonpad * has * n,
                            m[3] * 100.0 / nonpad * has * n, n])
        self.acc += step
        self.last = (loss, metrics)

    def read(self):
        """dict(loss, top1, top5 running averages, loss_val = the last step's loss, count)."""
        s = self.acc.cpu().tolist()
        n = s[3]
        out = dict(loss=s[0] / n if n else 0.0, top1=s[1] / n if n else 0.0, top5=s[2] / n if n else 0.0, count=n)
        out["loss_val"] = float(self.last[0].detach().cpu()) if self.last is not None else 0.0
        return out
