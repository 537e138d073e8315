"""Deferred bf16 backward, phase-2 workspace of bad runs against a good run, mapped to the carve regions of this
shape (GPU diagnosis; tools/debug_ws_diff.py's setup).  dhg rows are (b, t): which BPTT step diverges first."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import sat_amd as sat  # noqa: E402
from oracle import sat_oracle as O  # noqa: E402

DEV = "cuda"
V, D, Lf, E, B, T = 60, 64, 16, 512, 3, 7
T1, R, HG = T - 1, B * (T - 1), 5 * E + D
p = O.make_decoder_params(V, D, E, True, 5)
rng = np.random.default_rng(5)
feats = torch.from_numpy(rng.standard_normal((B, Lf, D)).astype(np.float32)).to(DEV).bfloat16()
caps = O.make_captions(B, T, V, 6).to(DEV)
dec = sat.Decoder(V, D, tf=True, ado=True, attention=True)
dec.load_state_dict(p, strict=True)
dec = dec.to(DEV).train()
dec.dropout_mask = torch.ones(B, T - 1, 512, dtype=torch.uint8, device=DEV)
REG = {"dhg": (917760, R * HG * 4), "dhg_t": (1106688, R * HG * 2), "dgated": (1201152, 2 * B * D * 4),
       "dh_rec0": (1202688, B * E * 4), "dc": (1454592, B * E * 4), "dWs_acc": (1460736, B * Lf * E * 4),
       "dv_acc": (1608192, B * E * 4), "de_all": (1614592, R * Lf * 4), "part": (1615872, 12300 * 4)}


def step():
    dec.zero_grad(set_to_none=True)
    dec.policy = sat.Policy(decoder_splits=[2, 2, 2, 2])
    dec.defer_recurrent_backward(True)
    preds, alphas = dec(feats, caps)
    sat.caption_loss(preds, alphas, caps)[0].backward()
    torch.cuda.synchronize()
    ws = dec._pending_bwd[4]
    dec.finish_backward()
    dec.defer_recurrent_backward(False)
    torch.cuda.synchronize()
    g = dec.attention.U.weight.grad.detach().clone()
    return g, ws.clone()


runs = [step() for _ in range(24)]
ref_g = runs[-1][0]
errs = [((g - ref_g).abs().max() / ref_g.abs().max()).item() for g, _ in runs]
good = [i for i, e in enumerate(errs) if e < 1e-5]
bad = [i for i, e in enumerate(errs) if e >= 1e-5]
print("bad runs", bad, "good runs", good[:4], flush=True)
if bad and good:
    gw = runs[good[0]][1]
    for i in bad[:3]:
        bw = runs[i][1]
        print(f"run {i}:")
        for name, (off, n) in REG.items():
            a = gw[off:off + n].view(torch.float32 if name != "dhg_t" else torch.bfloat16).float()
            b = bw[off:off + n].view(torch.float32 if name != "dhg_t" else torch.bfloat16).float()
            d = (a - b).abs()
            if name in ("dhg", "dhg_t"):
                rows = d.view(B, T1, HG).amax(dim=2)   # [b][t]
                print(f"  {name}: max diff per (b, t):", [[f"{x:.1e}" for x in r] for r in rows.tolist()])
                cols = d.view(R, HG).amax(dim=0)
                print(f"  {name}: max diff per column block [dUh | dfbeta | i f g o]:",
                      [f"{cols[s:e].max().item():.1e}" for s, e in ((0, E), (E, E + D), (E + D, 2 * E + D),
                                                                     (2 * E + D, 3 * E + D), (3 * E + D, 4 * E + D),
                                                                     (4 * E + D, 5 * E + D))])
            else:
                print(f"  {name}: max diff {d.max().item():.2e} (max |good| {a.abs().max().item():.2e})")
