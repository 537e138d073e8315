"""Debug helper: sweep decoder configs against the oracle (eval forward)."""
import itertools
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import sat_amd
from oracle import sat_oracle as O

dev = "cuda"
for bert, ado, att, tf, E in itertools.product([False, True], [True, False], [False, True], [False, True], [512, 768]):
    if bert and E != 768:
        continue
    if not bert and E != 512:
        continue
    B, L, D, V, T = 2, 16, 32, 128, 6
    p = O.make_decoder_params(V, D, E, ado, 11)
    kw = dict(tf=tf, ado=ado, bert=bert, attention=att)
    dec = sat_amd.Decoder(V, D, bert_embedding_weight=p["embedding.weight"], **kw) if bert else sat_amd.Decoder(V, D, **kw)
    dec.load_state_dict(p)
    dec = dec.to(dev).eval()
    feats = torch.randn(B, L, D)
    caps = O.make_captions(B, T, V, 3, bert=bert)
    with torch.no_grad():
        preds, alphas = dec(feats.to(dev), caps.to(dev))
    rp, ra, _ = O.decoder_forward(p, feats, caps, tf=tf, ado=ado, attention=att, bert=bert)
    e = ((preds.cpu() - rp).abs().max() / rp.abs().max()).item()
    e0 = ((preds.cpu()[:, 0] - rp[:, 0]).abs().max() / rp.abs().max()).item()
    print(f"bert={bert} ado={ado} att={att} tf={tf} E={E}: rel {e:.2e} step0 {e0:.2e}", flush=True)
