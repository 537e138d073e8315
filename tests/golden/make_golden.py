"""Generate golden vectors by running the REFERENCE decoder in this container.

Run (build container only; /root/reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference's ``attention.py`` / ``decoder.py`` are imported read-only from
``/root/reference`` (nothing is written there: bytecode writing is disabled),
with ``decoder.mps_device`` pointed at the CPU (the module global is otherwise
undefined off-Mac, decoder.py:5-6).  For ``bert=True`` the two
``from_pretrained`` classmethods are patched before ``Decoder`` is built so no
download happens: a locally built, 1-layer ``BertModel`` with a small vocabulary
stands in (the decoder only keeps its ``get_input_embeddings()`` table, which
we overwrite via ``load_state_dict`` anyway) and a stub tokenizer supplies the
ids the decoder reads (cls 101).

Weights are NOT stored: they are regenerated from a seed by
``oracle.sat_oracle.make_decoder_params`` (numpy PCG64, platform-stable) and
loaded into the reference module.  Each ``.npz`` holds inputs, full outputs,
and for gradients / post-Adam parameters a fixed sample of entries plus
per-tensor sums and sums of squares, which keeps every file well under 1 MB.
"""
import json
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import sat_oracle as O  # noqa: E402

REF = "/root/reference"

CONFIGS = [
    # name,                tf,    ado,   att,   bert,  B, L,  D,  V,   T
    ("att_tf_ado",         True,  True,  True,  False, 3, 16, 64, 60,  9),
    ("att_tf_simple",      True,  False, True,  False, 3, 16, 64, 60,  9),
    ("att_greedy_ado",     False, True,  True,  False, 3, 16, 64, 60,  9),
    ("att_greedy_simple",  False, False, True,  False, 2, 12, 48, 50,  8),
    ("noatt_tf_ado",       True,  True,  False, False, 3, 16, 64, 60,  9),
    ("noatt_greedy_simple", False, False, False, False, 2, 12, 48, 50, 8),
    ("bert_att_tf_simple", True,  False, True,  True,  2, 16, 32, 128, 10),
    ("bert_noatt_greedy_ado", False, True, False, True, 2, 16, 32, 128, 10),
]
SAMPLES = 48
LR = 1e-3
ALPHA_C = 1.0


def import_reference():
    sys.path.insert(0, REF)
    import attention as ref_attention  # noqa: F401
    import decoder as ref_decoder
    ref_decoder.mps_device = torch.device("cpu")
    sys.path.remove(REF)
    return ref_decoder


class _StubTok:
    cls_token_id = 101
    sep_token_id = 102
    pad_token_id = 0


def patch_bert(V):
    import transformers
    from transformers import BertConfig, BertModel

    def fake_model(*a, **k):
        return BertModel(BertConfig(vocab_size=V, hidden_size=768, num_hidden_layers=1,
                                    num_attention_heads=12, intermediate_size=64))

    transformers.BertModel.from_pretrained = staticmethod(fake_model)
    transformers.BertTokenizer.from_pretrained = staticmethod(lambda *a, **k: _StubTok())


class MaskDropout(torch.nn.Module):
    """Replaces nn.Dropout(): applies the pre-drawn mask of the current step."""

    def __init__(self, masks):
        super().__init__()
        self.masks = masks
        self.i = 0

    def forward(self, x):
        if not self.training:
            return x
        m = self.masks[self.i]
        self.i += 1
        return x * m * 2.0


def sample_idx(numel, name):
    rng = np.random.default_rng(abs(hash(name)) % (2 ** 32) if False else 1000 + numel)
    return np.sort(rng.choice(numel, size=min(SAMPLES, numel), replace=False))


def main():
    ref_decoder = import_reference()
    torch.manual_seed(0)
    for (name, tf, ado, att, bert, B, L, D, V, T) in CONFIGS:
        if bert:
            patch_bert(V)
        E = 768 if bert else 512
        seed = 7 + len(name)
        dec = ref_decoder.Decoder(V, D, tf=tf, ado=ado, bert=bert, attention=att)
        params = O.make_decoder_params(V, D, E, ado, seed)
        dec.load_state_dict(params, strict=True)
        rng = np.random.default_rng(seed + 1)
        feats = torch.from_numpy(rng.standard_normal((B, L, D)).astype(np.float32))
        caps = O.make_captions(B, T, V, seed + 2, bert=bert)
        out = {"meta": np.array(json.dumps(dict(name=name, tf=tf, ado=ado, attention=att, bert=bert,
                                                B=B, L=L, D=D, V=V, T=T, E=E, seed=seed,
                                                lr=LR, alpha_c=ALPHA_C))),
               "img_features": feats.numpy(), "captions": caps.numpy()}
        # --- eval-mode forward -------------------------------------------------
        dec.eval()
        with torch.no_grad():
            h0, c0 = dec.get_init_lstm_state(feats)
            out["h0"], out["c0"] = h0.numpy(), c0.numpy()
            if att:
                ctx, alpha = dec.attention(feats, h0)
                out["att_context"], out["att_alpha"] = ctx.numpy(), alpha.numpy()
            preds, alphas = dec(feats, caps)
            out["eval_preds"], out["eval_alphas"] = preds.numpy(), alphas.numpy()
            out["eval_ids"] = preds.max(2)[1].numpy()
            out["eval_top2_gap"] = (preds.topk(2, dim=2)[0][..., 0] - preds.topk(2, dim=2)[0][..., 1]).numpy()
            out["eval_loss"] = np.float32(O.caption_loss(preds, alphas, caps, ALPHA_C).item())
            pad = 0 if bert else 3
            out["acc1"] = np.float64(O.sequence_accuracy(preds, caps[:, 1:], 1, pad))
            out["acc5"] = np.float64(O.sequence_accuracy(preds, caps[:, 1:], 5, pad))
            skip = [0, 101, 102] if bert else [3, 0, 1]
            out["caption_length"] = np.int64(O.calculate_caption_lengths(caps, skip))
        # --- train-mode step with injected dropout masks ----------------------
        masks = O.make_dropout_masks(B, T - 1, E, seed + 3)
        dec.train()
        dec.dropout = MaskDropout(masks)
        opt = torch.optim.Adam(dec.parameters(), lr=LR)
        opt.zero_grad()
        preds, alphas = dec(feats, caps)
        targets = caps[:, 1:]
        packed_targets = torch.nn.utils.rnn.pack_padded_sequence(targets, [len(t) - 1 for t in targets], batch_first=True)[0]
        packed_preds = torch.nn.utils.rnn.pack_padded_sequence(preds, [len(p) - 1 for p in preds], batch_first=True)[0]
        att_reg = ALPHA_C * ((1 - alphas.sum(1)) ** 2).mean()
        loss = torch.nn.CrossEntropyLoss()(packed_preds, packed_targets) + att_reg
        loss.backward()
        out["train_loss"] = np.float32(loss.item())
        out["train_preds"] = preds.detach().numpy()
        out["train_alphas"] = alphas.detach().numpy()
        grad_names = []
        for pname, prm in dec.named_parameters():
            if prm.grad is None:
                continue
            grad_names.append(pname)
            g = prm.grad.detach().reshape(-1).double().numpy()
            idx = sample_idx(g.size, pname)
            out[f"gidx::{pname}"] = idx
            out[f"gval::{pname}"] = g[idx].astype(np.float32)
            out[f"gsum::{pname}"] = np.float64(g.sum())
            out[f"gsq::{pname}"] = np.float64((g * g).sum())
        out["grad_names"] = np.array(json.dumps(grad_names))
        opt.step()
        for pname, prm in dec.named_parameters():
            if pname in grad_names:
                w = prm.detach().reshape(-1).numpy()
                out[f"pval::{pname}"] = w[out[f"gidx::{pname}"]]
        path = os.path.join(HERE, f"decoder_{name}.npz")
        np.savez_compressed(path, **out)
        print(f"{path}: {os.path.getsize(path) / 1024:.1f} KB, loss={out['train_loss']:.6f}")

    # VGG19 layer / parameter table printed by nb_tests.ipynb (cells 0 and 6).
    nb = json.load(open(os.path.join(REF, "nb_tests.ipynb")))
    table = []
    for o in nb["cells"][6].get("outputs", []):
        text = "".join(o.get("text", []))
        for line in text.splitlines():
            parts = [p.strip() for p in line.strip("|").split("|")]
            if len(parts) == 2 and parts[0].startswith("features.") and parts[1].isdigit():
                table.append([parts[0], int(parts[1])])
    with open(os.path.join(HERE, "vgg19_param_table.json"), "w") as f:
        json.dump({"source": "nb_tests.ipynb cell 6 output (features.* rows)", "rows": table}, f, indent=0)
    print("vgg19 rows:", len(table))


if __name__ == "__main__":
    main()
