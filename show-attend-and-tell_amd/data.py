"""Synthetic inputs in the reference's data layout.

Images: the post-Normalize domain of train.py:27-32, i.e. [B,3,224,224] f32 ~ N(0,1).
Plain captions ``<start>=0 w.. <eos>=1 <pad>=3..`` (generate_json_data.py:71-78),
n ~ U{8..T-2}, words ~ U[4,V).  BERT captions ``[CLS]=101 w.. [PAD]=0.. [SEP]=102``
(generate_json_data_bert.py:44-47; SEP after the padding, as the reference writes it).
"""
import torch


def synthetic_captions(B, T, V, generator=None, bert=False, device="cpu"):
    g = generator
    body = T - 2
    if bert:
        n = torch.randint(1, body + 1, (B,), generator=g)
        words = torch.randint(min(1000, V - 1), V, (B, body), generator=g)
        pos = torch.arange(body).unsqueeze(0)
        body_t = torch.where(pos < n.unsqueeze(1), words, torch.zeros_like(words))
        caps = torch.cat([torch.full((B, 1), 101), body_t, torch.full((B, 1), 102)], 1)
    else:
        n = torch.randint(min(8, body), body + 1, (B,), generator=g)
        words = torch.randint(4, V, (B, body + 1), generator=g)
        pos = torch.arange(body + 1).unsqueeze(0)
        ln = n.unsqueeze(1)
        body_t = torch.where(pos < ln, words, torch.where(pos == ln, torch.ones_like(words), torch.full_like(words, 3)))
        caps = torch.cat([torch.zeros(B, 1, dtype=torch.long), body_t], 1)
    return caps.long().to(device)


def synthetic_images(B, H=224, W=224, generator=None, device="cpu"):
    return torch.randn(B, 3, H, W, generator=generator).to(device)
