"""Diagnostics: the greedy decoder step's two forms (SatPolicy.greedy_step 0 fused / 1 per-op) in training mode with
seeded or injected dropout, repeated, against the bf16 rounding mirror of the oracle conditioned on the fed tokens.
Prints per-form relative errors (preds, loss, per-parameter gradient norms) and run-to-run gradient differences."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402

import sat_amd as sat  # noqa: E402
from oracle import sat_oracle as O  # noqa: E402
import test_gpu_shapes as S  # noqa: E402
import test_gpu_greedy as G  # noqa: E402


def run(form, ado, inject, seed_case=23):
    D, Lf, E, V, T = 512, 196, 512, 2600, 8
    c = S._make_case(D, Lf, E, V, T, False, ado, False, 4, seed_case)
    dec = S._decoder(sat, c).train()
    dec.policy = sat.Policy(greedy_step=form)
    if inject:
        dec._seed_host = 12345
        m = G.host_dropout_masks(12345, 4, T - 1, E)
        dec.dropout_mask = m.permute(1, 0, 2).contiguous().to(torch.uint8)
    caps = c["caps"].to("cuda")
    preds, alphas = dec(c["feats"].to("cuda").bfloat16(), caps)
    pad, skip = sat.special_ids(False)
    loss, _ = sat.caption_loss(preds, alphas, caps, 1.0, pad, skip)
    loss.backward()
    torch.cuda.synchronize()
    params = dict(dec.named_parameters())
    grads = {n: params[n].grad.detach().float().cpu().clone() for n in dec.active_param_names()}
    h = dict(loss=loss.item(), preds=preds.detach().float().cpu(), alphas=alphas.detach().float().cpu(),
             grads=grads, tokens=dec.last_tokens.long().cpu())
    c = dict(c, masks=G.host_dropout_masks(dec._seed_host, 4, T - 1, E))
    with O.bf16_mirror():
        loss_f, g_f, _, preds_f, _ = S._oracle_fed(c, h["tokens"], torch.float64)
    errs = S._grad_errors(h, {n: g.float() for n, g in g_f.items()})
    print(f"form {form} ado {ado} inject {inject}: preds {S.rel(h['preds'], preds_f):.2e} "
          f"loss {abs(h['loss'] - loss_f.item()) / abs(loss_f.item()):.2e} max grad err "
          f"{max(errs.values()):.4f} ({max(errs, key=errs.get)})", flush=True)
    return h


for ado in (True, False):
    for inject in (False, True):
        for form in (1, 0):
            hs = [run(form, ado, inject) for _ in range(3)]
            for n in hs[0]["grads"]:
                d = max((h["grads"][n] - hs[0]["grads"][n]).abs().max().item() for h in hs[1:])
                if d != 0:
                    print(f"   run-to-run difference {n}: {d:.3e}")
