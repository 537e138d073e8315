"""Host-side logic that needs no GPU: module API / state_dict contract against the reference
layout, the flat parameter buffer, synthetic data layout, and that the product path refuses
CPU tensors (no silent fallback)."""
import pytest
import torch

import sat_amd
from oracle import sat_oracle as O


@pytest.mark.parametrize("ado", [False, True])
@pytest.mark.parametrize("attention", [False, True])
def test_decoder_state_dict_contract(ado, attention):
    dec = sat_amd.Decoder(100, 64, tf=True, ado=ado, attention=attention)
    sd = dec.state_dict()
    ref = O.decoder_param_shapes(100, 64, 512, ado)
    assert list(sd.keys()) == [k for k, _ in ref]
    for k, shape in ref:
        assert tuple(sd[k].shape) == shape
    for attr in ("use_tf", "use_advanced_deep_output", "use_bert", "use_attention", "vocabulary_size",
                 "embedding_size", "encoder_dim"):
        assert hasattr(dec, attr)


def test_bert_decoder_contract():
    emb = torch.randn(128, 768)
    dec = sat_amd.Decoder(0, 32, bert=True, bert_embedding_weight=emb)
    assert dec.vocabulary_size == 128 and dec.embedding_size == 768
    assert not dec.embedding.weight.requires_grad
    assert dec.tokenizer.cls_token_id == 101
    assert "embedding.weight" not in dec.active_param_names()


def test_flat_buffer_layout_and_aliasing():
    torch.manual_seed(0)
    dec = sat_amd.Decoder(100, 64, tf=True, ado=True, attention=True)
    before = {k: v.clone() for k, v in dec.state_dict().items()}
    dec._build_flat(torch.device("cpu"))
    o, E, D = dec._offsets, 512, 64
    assert o["init_c.weight"] == o["init_h.weight"] + E * D
    assert o["init_c.bias"] == o["init_h.bias"] + E
    assert o["f_beta.weight"] == o["attention.U.weight"] + E * E
    assert o["lstm.weight_hh"] == o["f_beta.weight"] + D * E
    assert o["f_beta.bias"] == o["attention.U.bias"] + E
    assert o["lstm.bias_hh"] == o["f_beta.bias"] + D
    assert all(off % 64 == 0 for n, off in o.items() if n in ("init_h.weight", "attention.U.weight", "lstm.weight_ih"))
    assert dec._flat_ok(torch.device("cpu"))
    for k, v in dec.state_dict().items():
        assert torch.equal(v, before[k])
    # load_state_dict copies in place: the aliasing survives
    dec.load_state_dict({k: torch.randn_like(v) for k, v in before.items()})
    assert dec._flat_ok(torch.device("cpu"))
    assert dec.grad_bucket(1).numel() == (o["f_z.bias"] + E) - o["f_out.weight"]


@pytest.mark.parametrize("network", ["vgg19", "resnet152"])
def test_encoder_state_dict_contract(network):
    enc = sat_amd.Encoder(network)
    ref = O.make_vgg19_params(0) if network == "vgg19" else O.make_resnet152_params(0)
    sd = enc.state_dict()
    assert sorted(sd.keys()) == sorted(ref.keys())
    for k in ref:
        assert sd[k].shape == ref[k].shape, k
    assert enc.dim == (512 if network == "vgg19" else 2048)
    assert all(not p.requires_grad for p in enc.parameters())
    with pytest.raises(NotImplementedError):
        sat_amd.Encoder("densenet161")


def test_product_path_refuses_cpu_tensors():
    dec = sat_amd.Decoder(50, 64, tf=True, attention=True)
    with pytest.raises(RuntimeError, match="HIP device"):
        dec(torch.randn(2, 4, 64), torch.zeros(2, 5, dtype=torch.long))
    with pytest.raises(RuntimeError, match="HIP device"):
        sat_amd.caption_loss(torch.randn(2, 4, 50), torch.rand(2, 4, 4), torch.zeros(2, 5, dtype=torch.long))
    enc = sat_amd.Encoder("vgg19")
    with pytest.raises(RuntimeError, match="HIP device"):
        enc(torch.randn(1, 3, 32, 32))


def test_synthetic_caption_layout():
    from sat_amd.data import synthetic_captions
    caps = synthetic_captions(16, 27, 10000, torch.Generator().manual_seed(0))
    assert caps.shape == (16, 27) and caps.dtype == torch.long
    assert (caps[:, 0] == 0).all()
    for row in caps.tolist():
        eos = row.index(1)
        assert all(t >= 4 for t in row[1:eos]) and all(t == 3 for t in row[eos + 1:])
        assert 8 <= eos - 1 <= 25
    bert = synthetic_captions(4, 32, 30522, torch.Generator().manual_seed(0), bert=True)
    assert (bert[:, 0] == 101).all() and (bert[:, -1] == 102).all()


def test_cli_flags_mirror_reference():
    """train.py:438-472 and generate_caption.py:153-160 flags parse with the reference defaults."""
    import importlib.util, os
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "show-attend-and-tell_amd")
    spec = importlib.util.spec_from_file_location("sat_train_cli", os.path.join(pkg, "train.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    a = m.parse([])
    assert (a.batch_size, a.epochs, a.lr, a.step_size, a.alpha_c, a.seed, a.log_interval) == (64, 10, 1e-4, 5, 1, 42, 100)
    assert (a.data, a.network, a.tf, a.ado, a.fraction, a.bert, a.attention, a.perform_test) == \
        ("data/coco", "vgg19", False, False, 1.0, False, False, True)
    a = m.parse(["--tf", "--ado", "--attention", "--network", "resnet152"])
    assert a.tf and a.ado and a.attention and a.network == "resnet152"
    spec = importlib.util.spec_from_file_location("sat_gen_cli", os.path.join(pkg, "generate_caption.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    with pytest.raises(SystemExit):
        g.main(["--img-path", "x.png", "--wandb-run", "a/b/c", "--wandb-model", "m"])


def test_stem_space_to_depth_equivalence():
    """The ResNet152 stem (7x7 / stride 2 / pad 3, encoder.py:13-17 conv1) equals the 4x4 /
    stride-1 conv over the 2x2 space-to-depth input with stem_weight_s2d weights (top/left pad 2,
    bottom/right pad 1), checked in fp64 with torch's CPU conv as the reference."""
    import torch.nn.functional as F
    from sat_amd.encoder import stem_weight_s2d
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 3, 20, 16, generator=g, dtype=torch.float64)
    w = torch.randn(5, 3, 7, 7, generator=g, dtype=torch.float64)
    ref = F.conv2d(x, w, stride=2, padding=3)
    N, C, H, W = x.shape
    xs = torch.zeros(N, 16, H // 2, W // 2, dtype=x.dtype)   # sat_nchw_to_s2d's channel order
    for sy in range(2):
        for sx in range(2):
            c0 = (sy * 2 + sx) * C
            xs[:, c0:c0 + C] = x[:, :, sy::2, sx::2]
    ws = stem_weight_s2d(w.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)
    out = F.conv2d(F.pad(xs, (2, 1, 2, 1)), ws)
    assert out.shape == ref.shape
    assert torch.allclose(out, ref, rtol=0, atol=1e-10)
