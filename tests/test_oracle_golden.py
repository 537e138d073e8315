"""Pin the CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py ran the reference decoder.py / attention.py)."""
import json
import math
import os

import numpy as np
import pytest
import torch

from golden_util import fixture_paths, fixture_ids, load, params_for, masks_for, t
from oracle import sat_oracle as O

RTOL = 1e-4  # north_star: 1e-4 relative on forward / loss


def rel(a, b):
    a = torch.as_tensor(a, dtype=torch.float64); b = torch.as_tensor(b, dtype=torch.float64)
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


@pytest.mark.parametrize("path", fixture_paths(), ids=fixture_ids())
def test_oracle_eval_forward(path):
    g = load(path); c = g["cfg"]
    p = params_for(c)
    feats, caps = t(g["img_features"]), t(g["captions"])
    h0, c0 = O.init_lstm_state(p, feats)
    assert rel(h0, g["h0"]) < RTOL and rel(c0, g["c0"]) < RTOL
    if c["attention"]:
        ctx, alpha = O.attention_forward(p, feats, h0)
        assert rel(ctx, g["att_context"]) < RTOL and rel(alpha, g["att_alpha"]) < RTOL
    preds, alphas, _ = O.decoder_forward(p, feats, caps, tf=c["tf"], ado=c["ado"], attention=c["attention"], bert=c["bert"])
    assert rel(preds, g["eval_preds"]) < RTOL
    assert rel(alphas, g["eval_alphas"]) < RTOL
    assert np.array_equal(preds.max(2)[1].numpy(), g["eval_ids"])  # greedy ids bit-exact
    loss = O.caption_loss(preds, alphas, caps, c["alpha_c"]).item()
    assert abs(loss - float(g["eval_loss"])) <= RTOL * abs(float(g["eval_loss"]))
    pad = 0 if c["bert"] else 3
    assert O.sequence_accuracy(preds, caps[:, 1:], 1, pad) == pytest.approx(float(g["acc1"]))
    assert O.sequence_accuracy(preds, caps[:, 1:], 5, pad) == pytest.approx(float(g["acc5"]))
    skip = [0, 101, 102] if c["bert"] else [3, 0, 1]
    assert O.calculate_caption_lengths(caps, skip) == int(g["caption_length"])


@pytest.mark.parametrize("path", fixture_paths(), ids=fixture_ids())
def test_oracle_train_step(path):
    g = load(path); c = g["cfg"]
    p = params_for(c)
    feats, caps = t(g["img_features"]), t(g["captions"])
    loss, grads, newp, preds, alphas = O.train_step(p, feats, caps, tf=c["tf"], ado=c["ado"], attention=c["attention"],
                                                    bert=c["bert"], alpha_c=c["alpha_c"], lr=c["lr"],
                                                    dropout_masks=masks_for(c))
    assert abs(loss.item() - float(g["train_loss"])) <= RTOL * abs(float(g["train_loss"]))
    assert rel(preds, g["train_preds"]) < RTOL
    assert sorted(grads) == sorted(g["grad_names"])
    for name in g["grad_names"]:
        gr = grads[name].reshape(-1).double()
        ref_norm = math.sqrt(float(g[f"gsq::{name}"]))
        idx = torch.from_numpy(g[f"gidx::{name}"])
        if ref_norm < 1e-7:   # attention.v.bias: analytically zero (softmax shift invariance)
            assert gr.abs().max().item() < 1e-6
            continue
        assert abs(gr.norm().item() - ref_norm) <= 1e-4 * ref_norm, name
        err = (gr[idx] - torch.from_numpy(g[f"gval::{name}"]).double()).abs().max().item()
        assert err <= 1e-4 * gr.abs().max().item() + 1e-9, name
        # post-Adam params: an Adam update is bounded by ~lr, so compare at lr scale
        w = newp[name].reshape(-1)[idx].double()
        assert (w - torch.from_numpy(g[f"pval::{name}"]).double()).abs().max().item() <= 1e-3 * c["lr"] + 1e-6, name


def test_vgg19_layer_table_matches_reference_notebook(golden_dir):
    rows = json.load(open(os.path.join(golden_dir, "vgg19_param_table.json")))["rows"]
    p = O.make_vgg19_params(0)
    ours = [[k.replace("net.", "features."), v.numel()] for k, v in p.items()]
    assert ours == rows


def test_resnet152_shapes_and_params():
    p = O.make_resnet152_params(0)
    n = sum(v.numel() for k, v in p.items() if not k.endswith("running_mean") and not k.endswith("running_var")
            and not k.endswith("num_batches_tracked"))
    assert n == 58143808   # torchvision resnet152 minus fc (2048*1000+1000) = 60192808 - 2049000
    x = torch.randn(1, 3, 64, 64)
    assert O.resnet152_forward(p, x).shape == (1, 4, 2048)
    assert O.vgg19_forward(O.make_vgg19_params(0), x).shape == (1, 16, 512)


@pytest.mark.parametrize("path", __import__("golden_util").beam_paths(), ids=__import__("golden_util").beam_ids())
def test_oracle_beam_search(path):
    """oracle.beam_search == reference Decoder.caption (decoder.py:160-269) on the golden cases."""
    from golden_util import load_beam
    g = load_beam(path)
    cfg = g["cfg"]
    with torch.no_grad():
        ids, al, score = O.beam_search(g["params"], g["feats"], cfg["beam"], ado=cfg["ado"],
                                       attention=cfg["attention"], bert=cfg["bert"])
    assert ids == g["sentence"].tolist()
    np.testing.assert_allclose(np.array(al, dtype=np.float32), g["alphas"], rtol=1e-5, atol=1e-6)
    if math.isinf(float(g["score"])):
        assert math.isinf(score)
    else:
        assert abs(score - float(g["score"])) <= 1e-5 * max(1.0, abs(score))


def test_greedy_equals_teacher_forcing_on_its_own_tokens():
    """The premise of the GPU greedy tests' conditioned oracle (test_gpu_shapes._oracle_fed): the greedy decoder
    (decoder.py:131-133, argmax fed back) is the teacher-forced decoder run on the tokens it fed itself -- same
    preds, alphas, loss against the real captions and gradients (the argmax is a constant for autograd)."""
    V, D, E, B, T = 40, 32, 512, 3, 7
    p = O.make_decoder_params(V, D, E, True, 3)
    feats = torch.randn(B, 9, D, generator=torch.Generator().manual_seed(4)).relu()
    caps = O.make_captions(B, T, V, 5)
    masks = O.make_dropout_masks(B, T - 1, E, 6)
    names = O.trainable_names(V, D, E, True, True, False)

    def run(tf, fed_caps):
        q = {k: v.clone().requires_grad_(k in names) for k, v in p.items()}
        preds, alphas, toks = O.decoder_forward(q, feats, fed_caps, tf=tf, ado=True, attention=True, training=True,
                                                dropout_masks=masks)
        loss = O.caption_loss(preds, alphas, caps)
        loss.backward()
        return preds.detach(), alphas.detach(), loss.item(), toks, {k: q[k].grad for k in names}
    pg, ag, lg, toks, gg = run(False, caps)
    fed = caps.clone()
    fed[:, :T - 1] = toks
    pt, at, lt, toks2, gt = run(True, fed)
    assert torch.equal(toks, toks2)
    assert torch.equal(pg, pt) and torch.equal(ag, at) and lg == lt
    for k in names:
        assert torch.equal(gg[k], gt[k]), k
