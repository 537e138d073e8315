"""Diagnostics: test_gpu_api.py::test_policy_edit_between_forward_and_deferred_backward's two steps repeated in one
process; prints, per repeat, the largest relative gradient difference between the plain and the edited-policy step
and between two plain steps (run-to-run), so a nondeterministic reduction shows up as a nonzero second column."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402

import sat_amd as sat  # noqa: E402
import test_gpu_api as A  # noqa: E402

dec, feats, caps = A._setup(sat)
feats = feats.bfloat16()
dec.train()
dec.dropout_mask = torch.ones(feats.shape[0], caps.shape[1] - 1, 512, dtype=torch.uint8, device="cuda")


EXTRA = dict(kv.split("=") for kv in sys.argv[2:])   # extra SatPolicy fields, e.g. attn_bwd_chunks=1
EXTRA = {k: int(v) for k, v in EXTRA.items()}


def step(edit):
    dec.zero_grad(set_to_none=True)
    dec.policy = sat.Policy(decoder_splits=[2, 2, 2, 2], **EXTRA)
    dec.defer_recurrent_backward(True)
    preds, alphas = dec(feats, caps)
    step.preds = preds.detach().float().clone()
    sat.caption_loss(preds, alphas, caps)[0].backward()
    step.phase1 = {n: p.grad.detach().clone() for n, p in dec.named_parameters() if p.grad is not None}
    if edit:
        dec.policy.decoder_splits[:] = [4, 4, 4, 4]
        dec.policy.attn_bwd_chunks = 3
    dec.finish_backward()
    dec.defer_recurrent_backward(False)
    torch.cuda.synchronize()
    return A._grads(dec)


def worst(a, b):
    out = {}
    for n in a:
        d = (a[n] - b[n]).abs().max().item()
        if d:
            out[n] = d / max(a[n].abs().max().item(), 1e-30)
    return out


ref = step(False)
ref_preds, ref_p1 = step.preds, step.phase1
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    p = step(False)
    dp = (step.preds - ref_preds).abs().max().item()
    w1 = worst(ref_p1, step.phase1)
    wp = worst(ref, p)
    top = sorted(wp.items(), key=lambda kv: -kv[1])[:4]
    print(i, f"preds {dp:.2e}", "phase1:", {k: f"{v:.1e}" for k, v in sorted(w1.items(), key=lambda kv: -kv[1])[:3]},
          "final:", {k: f"{v:.1e}" for k, v in top}, flush=True)
