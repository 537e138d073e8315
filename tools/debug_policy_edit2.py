"""Which runs of the deferred two-phase bf16 backward differ (GPU diagnosis): 12 runs per variant, each compared with
run 11 (the last), per-parameter relative max difference of the largest offenders."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import sat_amd as sat  # noqa: E402
from oracle import sat_oracle as O  # noqa: E402

DEV = "cuda"
V, D, Lf, E, B, T = 60, 64, 16, 512, 3, 7
p = O.make_decoder_params(V, D, E, True, 5)
rng = np.random.default_rng(5)
feats = torch.from_numpy(rng.standard_normal((B, Lf, D)).astype(np.float32)).to(DEV).bfloat16()
caps = O.make_captions(B, T, V, 6).to(DEV)
dec = sat.Decoder(V, D, tf=True, ado=True, attention=True)
dec.load_state_dict(p, strict=True)
dec = dec.to(DEV).train()
dec.dropout_mask = torch.ones(B, T - 1, 512, dtype=torch.uint8, device=DEV)


def step(kw, defer):
    dec.zero_grad(set_to_none=True)
    dec.policy = sat.Policy(**kw)
    dec.defer_recurrent_backward(defer)
    preds, alphas = dec(feats, caps)
    sat.caption_loss(preds, alphas, caps)[0].backward()
    dec.finish_backward()
    dec.defer_recurrent_backward(False)
    torch.cuda.synchronize()
    return {n: q.grad.detach().clone() for n, q in dec.named_parameters() if q.grad is not None}, preds.detach().clone()


NAMES = ("attention.U.weight", "init_h.weight", "lstm.weight_hh", "f_h.weight", "f_out.weight", "f_z.weight",
         "f_h.bias", "embedding.weight")
for label, kw, defer in [("splits2", dict(decoder_splits=[2, 2, 2, 2]), False)]:
    runs = [step(kw, defer) for _ in range(24)]
    ref, pref = runs[-1]
    line = []
    for i, (g, pr) in enumerate(runs[:-1]):
        d = {n: ((g[n] - ref[n]).abs().max() / ref[n].abs().max()).item() for n in NAMES}
        n_w = max(d, key=d.get)
        line.append(f"{i}:{d[n_w]:.1e}" + (f"({n_w.split('.')[0]})" if d[n_w] > 1e-5 else "") +
                    ("P" if not torch.equal(pr, pref) else ""))
    print(label, " ".join(line), flush=True)
