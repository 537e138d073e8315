import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, sat_amd
from oracle import sat_oracle as O
dev = "cuda"
B, L, D, V, T, E = 2, 16, 32, 128, 6, 768
p = O.make_decoder_params(V, D, E, False, 11)
dec = sat_amd.Decoder(V, D, tf=False, bert=True, bert_embedding_weight=p["embedding.weight"])
print("tokenizer", type(dec.tokenizer), dec.tokenizer.cls_token_id)
dec.load_state_dict(p); dec = dec.to(dev).eval()
feats = torch.randn(B, L, D); caps = O.make_captions(B, T, V, 3, bert=True)
with torch.no_grad():
    preds, _ = dec(feats.to(dev), caps.to(dev))
print("fed tokens", dec.last_tokens.cpu().tolist())
O.SPECIAL_BERT["start"] = 101
rp, _, tok = O.decoder_forward(p, feats, caps, tf=False, ado=False, attention=False, bert=True)
print("oracle tokens", tok.tolist(), ((preds.cpu() - rp).abs().max() / rp.abs().max()).item())
d = dec._dims(feats.to(dev).float(), caps.to(dev)); print("dims start", d.start_token, d.bert, d.tf, d.E)
