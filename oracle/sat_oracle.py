"""CPU oracle for the Show-Attend-and-Tell training hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker / the
CPU baseline.  The product path (``sat_amd``) never imports it and fails loudly
when its HIP library is missing.

This is a plain torch-CPU fp32 restatement of the reference algorithm
(yvokeller/Show-Attend-and-Tell @ v1), written from the reference behaviour,
one function per reference entry point, each citing the file:line it follows.
It is pinned against golden vectors produced by running the reference's own
``attention.py`` / ``decoder.py`` in the build container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``); the pinning test is
``tests/test_oracle_golden.py``.  The encoder trunks restate torchvision 0.16
(absent from the image) and are pinned by the layer/parameter table the
reference notebook prints (``nb_tests.ipynb`` cells 0 and 6), stored as
``tests/golden/vgg19_param_table.json``.  ``corpus_bleu`` restates nltk 3.8.1
(absent) and is pinned by hand-computed known-answer tests only
("parity unpinned" against nltk itself).

Parameters are passed as a flat ``dict`` keyed exactly like the reference
``Decoder.state_dict()``.
"""
from __future__ import annotations

import math
import sys
from collections import Counter
from fractions import Fraction

import numpy as np
import torch
import torch.nn.functional as F

# ----------------------------------------------------------------------------
# Deterministic parameter / input generation (shared by fixtures and tests).
# numpy's PCG64 stream is stable across platforms, so the same seed gives the
# same weights here and on the GPU box without shipping the weights.
# ----------------------------------------------------------------------------

SPECIAL_PLAIN = dict(start=0, eos=1, unk=2, pad=3)          # generate_json_data.py:45-48
SPECIAL_BERT = dict(start=101, eos=102, pad=0)               # [CLS]/[SEP]/[PAD]


def decoder_param_shapes(V: int, D: int, E: int, ado: bool):
    """Shapes of every decoder parameter, in reference state_dict order
    (decoder.py:10-67 construction order)."""
    s = [("embedding.weight", (V, E)),
         ("init_h.weight", (E, D)), ("init_h.bias", (E,)),
         ("init_c.weight", (E, D)), ("init_c.bias", (E,)),
         ("f_beta.weight", (D, E)), ("f_beta.bias", (D,)),
         ("attention.U.weight", (E, E)), ("attention.U.bias", (E,)),
         ("attention.W.weight", (E, D)), ("attention.W.bias", (E,)),
         ("attention.v.weight", (1, E)), ("attention.v.bias", (1,)),
         ("lstm.weight_ih", (4 * E, E + D)), ("lstm.weight_hh", (4 * E, E)),
         ("lstm.bias_ih", (4 * E,)), ("lstm.bias_hh", (4 * E,))]
    if ado:
        s += [("f_h.weight", (E, E)), ("f_h.bias", (E,)),
              ("f_z.weight", (E, D)), ("f_z.bias", (E,)),
              ("f_out.weight", (V, E)), ("f_out.bias", (V,))]
    s += [("deep_output.weight", (V, E)), ("deep_output.bias", (V,))]
    return s


def make_decoder_params(V, D, E, ado, seed, scale=1.0):
    """Uniform(-k, k) with k = 1/sqrt(fan_in) (torch Linear/LSTMCell default
    bound), embedding ~ N(0, 1) like nn.Embedding; deterministic from seed."""
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in decoder_param_shapes(V, D, E, ado):
        if name == "embedding.weight":
            a = rng.standard_normal(shape).astype(np.float32)
        else:
            if name.startswith("lstm."):
                fan_in = E
            elif name.endswith("bias"):
                fan_in = {"init_h.bias": D, "init_c.bias": D, "f_beta.bias": E,
                          "attention.U.bias": E, "attention.W.bias": D,
                          "attention.v.bias": E, "f_h.bias": E, "f_z.bias": D,
                          "f_out.bias": E, "deep_output.bias": E}[name]
            else:
                fan_in = shape[1]
            k = scale / math.sqrt(fan_in)
            a = rng.uniform(-k, k, size=shape).astype(np.float32)
        out[name] = torch.from_numpy(a)
    return out


def make_captions(B, T, V, seed, bert=False, min_len=None):
    """Synthetic padded captions in the reference layout:
    plain  ``<start> w.. <eos> <pad>..`` (generate_json_data.py:71-78);
    bert   ``[CLS] w.. [PAD].. [SEP]`` (generate_json_data_bert.py:44-47)."""
    rng = np.random.default_rng(seed)
    caps = np.zeros((B, T), dtype=np.int64)
    for b in range(B):
        if bert:
            body = T - 2
            n = int(rng.integers(1, body + 1))
            lo = min(1000, V - 1) if V > 1000 else 103
            toks = rng.integers(lo, V, size=n)
            caps[b] = [SPECIAL_BERT["start"]] + list(toks) + [SPECIAL_BERT["pad"]] * (body - n) + [SPECIAL_BERT["eos"]]
        else:
            body = T - 2
            lo_len = min_len if min_len is not None else max(1, min(8, body))
            n = int(rng.integers(lo_len, body + 1))
            toks = rng.integers(4, V, size=n)
            caps[b] = [SPECIAL_PLAIN["start"]] + list(toks) + [SPECIAL_PLAIN["eos"]] + [SPECIAL_PLAIN["pad"]] * (body - n)
    return torch.from_numpy(caps)


def make_dropout_masks(B, steps, E, seed):
    """Pre-drawn Bernoulli(0.5) keep-masks for train-mode parity (one per
    decoder step, as nn.Dropout() is called once per step, decoder.py:118-125)."""
    rng = np.random.default_rng(seed)
    return torch.from_numpy((rng.random((steps, B, E)) >= 0.5).astype(np.float32))


# ----------------------------------------------------------------------------
# Attention / decoder (attention.py, decoder.py)
# ----------------------------------------------------------------------------

# ----------------------------------------------------------------------------
# bf16 rounding mirror (test infrastructure): the HIP performance mode keeps bf16 copies of the weights and of the
# GEMM operands and accumulates in fp32.  Inside ``bf16_mirror()`` the decoder below rounds exactly there -- every
# Linear's input and weight (x, W -> bf16 values; the product and the bias add exact in the caller's dtype), the
# outputs the HIP path stores in bf16 (Ws = a W^T + b, attention.py:16, and the vocabulary logits, decoder.py:125 /
# 157), the embedding rows the ado combine adds (decoder.py:156), and in backward the gradient entering every such
# product (the HIP path stores it in bf16 before its input- and weight-gradient GEMMs; the bias gradients of the
# output-head Linears are column sums of those bf16 values, the others of the fp32 ones).  Everything else (the
# attention softmax / context, the gates, the LSTM cell, h, c, the loss) stays in the caller's dtype.  Run in fp64,
# it is the reference the bf16 kernels are measured against with fp32 accumulation noise as the only difference.
# ----------------------------------------------------------------------------

class _MirrorState:
    on = False


_MIRROR = _MirrorState()


class bf16_mirror:
    """Context manager: the decoder functions of this module round where the HIP bf16 path rounds."""

    def __enter__(self):
        self.prev = _MIRROR.on
        _MIRROR.on = True
        return self

    def __exit__(self, *exc):
        _MIRROR.on = self.prev
        return False


def _bf(x):
    return x.to(torch.bfloat16).to(x.dtype)


def _rb(x):
    """x rounded to bf16 values (same dtype) with a straight-through gradient."""
    return x + (_bf(x) - x).detach()


class _BF16Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, round_out, round_bias_grad):
        xr, wr = _bf(x), _bf(w)
        ctx.save_for_backward(xr, wr)
        ctx.rbg = round_bias_grad
        ctx.has_b = b is not None
        y = F.linear(xr, wr, b)
        return _bf(y) if round_out else y

    @staticmethod
    def backward(ctx, g):
        xr, wr = ctx.saved_tensors
        gr = _bf(g)
        dx = gr @ wr
        g2 = gr.reshape(-1, gr.shape[-1])
        dw = g2.T @ xr.reshape(-1, xr.shape[-1])
        db = None
        if ctx.has_b:
            db = (gr if ctx.rbg else g).reshape(-1, g.shape[-1]).sum(0)
        return dx, dw, db, None, None


def _lin(x, w, b, round_out=False, round_bias_grad=False, mirror=True):
    if mirror and _MIRROR.on:
        return _BF16Linear.apply(x, w, b, round_out, round_bias_grad)
    return F.linear(x, w, b)


# Linears whose output the HIP bf16 path stores in bf16, and those whose bias gradient is a column sum of a bf16
# gradient (the output head's)
_ROUND_OUT = ("attention.W", "f_out", "deep_output")
_ROUND_BIAS_GRAD = ("f_h", "f_z", "f_out", "deep_output")


def linear(x, p, name, mirror=True):
    return _lin(x, p[name + ".weight"], p[name + ".bias"], round_out=any(name.endswith(k) for k in _ROUND_OUT),
                round_bias_grad=name in _ROUND_BIAS_GRAD, mirror=mirror)


def attention_forward(p, img_features, hidden_state, prefix="attention."):
    """attention.py:14-21  e = v(tanh(W a + U h)); alpha = softmax_L(e);
    context = sum_l alpha_l a_l."""
    U_h = linear(hidden_state, p, prefix + "U").unsqueeze(1)
    W_s = linear(img_features, p, prefix + "W")
    att = torch.tanh(W_s + U_h)
    e = linear(att, p, prefix + "v", mirror=False).squeeze(2)   # fp32 weights in the HIP attention kernel
    alpha = torch.softmax(e, dim=1)
    context = (img_features * alpha.unsqueeze(2)).sum(1)
    return context, alpha


def init_lstm_state(p, img_features):
    """decoder.py:137-147"""
    avg = img_features.mean(dim=1)
    c = torch.tanh(linear(avg, p, "init_c"))
    h = torch.tanh(linear(avg, p, "init_h"))
    return h, c


def lstm_cell(p, x, h, c):
    """torch.nn.LSTMCell (decoder.py:53,115): gate order (i, f, g, o)."""
    g = _lin(x, p["lstm.weight_ih"], p["lstm.bias_ih"]) + _lin(h, p["lstm.weight_hh"], p["lstm.bias_hh"])
    i, f, gg, o = g.chunk(4, dim=1)
    c2 = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
    h2 = torch.sigmoid(o) * torch.tanh(c2)
    return h2, c2


def advanced_deep_output(p, h, context, emb):
    """decoder.py:149-158 (ungated context, ReLU on the logits)."""
    ht = torch.relu(linear(h, p, "f_h"))
    zt = torch.relu(linear(context, p, "f_z"))
    if _MIRROR.on:
        emb = _rb(emb)   # the bf16 embedding rows of the HIP combine
    return torch.relu(linear(ht + zt + emb, p, "f_out"))


def decoder_forward(p, img_features, captions, *, tf, ado, attention, bert=False,
                    training=False, dropout_masks=None):
    """decoder.py:69-135.  Returns (preds[B,T-1,V], alphas[B,T-1,L], in_tokens[B,T-1]).

    ``in_tokens[:, t]`` is the token whose embedding is fed at step t (the
    caption token under teacher forcing, the previous greedy argmax
    otherwise; decoder.py:87,131-133).  ``dropout_masks[t]`` replaces the
    Bernoulli draw of ``nn.Dropout()`` at step t when ``training``."""
    B, L, D = img_features.shape
    V = p["embedding.weight"].shape[0]
    emb_w = p["embedding.weight"]
    h, c = init_lstm_state(p, img_features)
    T1 = captions.shape[1] - 1                                    # decoder.py:77
    start = SPECIAL_BERT["start"] if bert else SPECIAL_PLAIN["start"]
    prev_tok = torch.full((B,), start, dtype=torch.long)           # decoder.py:79-82
    preds = torch.zeros(B, T1, V, dtype=img_features.dtype)
    alphas = torch.zeros(B, T1, L, dtype=img_features.dtype)
    in_tokens = torch.zeros(B, T1, dtype=torch.long)

    def dropout(x, t):
        if not training:
            return x
        if dropout_masks is None:
            return F.dropout(x, 0.5, True)
        return x * dropout_masks[t] * 2.0

    for t in range(T1):                                            # decoder.py:96
        tok = captions[:, t] if tf else prev_tok
        in_tokens[:, t] = tok
        emb = F.embedding(tok, emb_w)
        if attention:                                              # decoder.py:97-100
            context, alpha = attention_forward(p, img_features, h)
            gate = torch.sigmoid(linear(h, p, "f_beta"))
            gated = gate * context
        else:                                                      # decoder.py:101-105
            alpha = torch.full((B, L), 1.0 / L)
            context = img_features.mean(dim=1)
            gated = context
        x = torch.cat((emb, gated), dim=1)                         # decoder.py:107-112
        h, c = lstm_cell(p, x, h, c)                               # decoder.py:115
        if ado:                                                    # decoder.py:117-125
            out = advanced_deep_output(p, dropout(h, t), context, emb)
        else:
            out = linear(dropout(h, t), p, "deep_output")
        preds[:, t] = out
        alphas[:, t] = alpha
        if not tf:                                                 # decoder.py:131-133
            prev_tok = out.max(1)[1]
    return preds, alphas, in_tokens


def beam_search(p, img_features, beam_size, *, ado, attention, bert=False, max_step=50):
    """decoder.py:160-269 (Decoder.caption).  img_features: [beam_size, L, D].

    Returns (sentence ids incl. the start token, alpha rows [len][L] incl. the leading ones row,
    score) for the best completed beam; ([0], last alpha rows, -inf) when none completed.  Scores
    are summed RAW logits (decoder.py:204); ties inside topk go to the lower flat index."""
    L = img_features.shape[1]
    V = p["embedding.weight"].shape[0]
    start = SPECIAL_BERT["start"] if bert else SPECIAL_PLAIN["start"]
    prev_words = torch.full((beam_size,), start, dtype=torch.long)       # decoder.py:166-169
    sentences = prev_words.unsqueeze(1)
    top_preds = torch.zeros(beam_size, 1)
    alphas = torch.ones(beam_size, 1, L)
    done, done_alpha, done_score = [], [], []
    h, c = init_lstm_state(p, img_features)
    feats = img_features
    step = 1
    while True:
        emb = F.embedding(prev_words, p["embedding.weight"])
        k = feats.shape[0]
        if attention:
            context, alpha = attention_forward(p, feats, h)
            gated = torch.sigmoid(linear(h, p, "f_beta")) * context
        else:
            alpha = torch.full((k, L), 1.0 / L)
            context = feats.mean(dim=1)
            gated = context
        h, c = lstm_cell(p, torch.cat((emb, gated), dim=1), h, c)
        out = advanced_deep_output(p, h, context, emb) if ado else linear(h, p, "deep_output")
        out = top_preds.expand_as(out) + out                             # decoder.py:204
        flat = out[0] if step == 1 else out.reshape(-1)
        # sorted top-k with ties to the lower index: stable sort on -value
        order = torch.sort(-flat, stable=True).indices[:k]
        top_vals, top_words = flat[order], order
        prev_idx, next_idx = top_words // V, top_words % V                  # decoder.py:210-211
        sentences = torch.cat((sentences[prev_idx], next_idx.unsqueeze(1)), dim=1)
        alphas = torch.cat((alphas[prev_idx], alpha[prev_idx].unsqueeze(1)), dim=1)
        ends = (1, 0) if bert else (1, 102)                                 # decoder.py:224-229
        incomplete = [i for i, w in enumerate(next_idx.tolist()) if w not in ends]
        complete = sorted(set(range(k)) - set(incomplete))
        for i in complete:
            done.append(sentences[i].tolist())
            done_alpha.append(alphas[i].tolist())
            done_score.append(float(top_vals[i]))
        if len(incomplete) == 0:
            break
        sentences, alphas = sentences[incomplete], alphas[incomplete]
        sel = prev_idx[incomplete]
        h, c, feats = h[sel], c[sel], feats[sel]
        top_preds = top_vals[incomplete].unsqueeze(1)
        prev_words = next_idx[incomplete]
        if step > max_step:
            break
        step += 1
    if not done:
        return [0], alpha.tolist(), float("-inf")
    best = done_score.index(max(done_score))
    return done[best], done_alpha[best], done_score[best]


# ----------------------------------------------------------------------------
# Loss, metrics, optimiser (train.py, utils.py, torch.optim.Adam)
# ----------------------------------------------------------------------------

def caption_loss(preds, alphas, captions, alpha_c=1.0):
    """train.py:135,150-162: time-major CE over the first T-2 steps (pads
    included, last step never scored) + alpha_c * mean((1 - sum_t alpha)^2)."""
    B, T1, V = preds.shape
    targets = captions[:, 1:]
    Tl = T1 - 1                                  # pack_padded_sequence lengths = T-2
    packed_preds = preds[:, :Tl].transpose(0, 1).reshape(-1, V)
    packed_targets = targets[:, :Tl].transpose(0, 1).reshape(-1)
    att_reg = alpha_c * ((1 - alphas.sum(1)) ** 2).mean()
    return F.cross_entropy(packed_preds, packed_targets) + att_reg


def sequence_accuracy(preds, targets, k, ignore_index=0):
    """utils.py:44-80 (top-k over V, pad-masked, all T-1 steps)."""
    _, topk = preds.topk(k, dim=2, largest=True, sorted=True)
    mask = targets.ne(ignore_index)
    correct = (topk.eq(targets.unsqueeze(-1).expand_as(topk)) * mask.unsqueeze(-1)).any(dim=2)
    n = mask.sum().item()
    return correct.float().sum().item() * 100.0 / n if n > 0 else 0


def calculate_caption_lengths(captions, skip_tokens):
    """utils.py:101-107"""
    skip = torch.as_tensor(skip_tokens)
    return int((~captions.unsqueeze(-1).eq(skip).any(-1)).sum().item())


def adam_step(params, grads, state, lr, betas=(0.9, 0.999), eps=1e-8):
    """torch.optim.Adam (train.py:71; defaults, no weight decay, no amsgrad),
    the single-tensor CPU algorithm:  m.lerp_(g, 1-b1); v = v*b2 + (1-b2) g^2;
    p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps).  Params whose grad is None are
    skipped (they keep no state)."""
    b1, b2 = betas
    for name, p in params.items():
        g = grads.get(name)
        if g is None:
            continue
        st = state.setdefault(name, {"step": 0, "m": torch.zeros_like(p), "v": torch.zeros_like(p)})
        st["step"] += 1
        st["m"].lerp_(g, 1 - b1)
        st["v"].mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** st["step"]
        bc2 = 1 - b2 ** st["step"]
        denom = (st["v"].sqrt() / math.sqrt(bc2)).add_(eps)
        p.addcdiv_(st["m"], denom, value=-(lr / bc1))
    return params


def trainable_names(V, D, E, ado, attention, bert):
    """Names whose grad is not None after loss.backward():
    unused head / attention params have no grad; BERT embeddings are frozen."""
    names = []
    for name, _ in decoder_param_shapes(V, D, E, ado):
        if bert and name == "embedding.weight":
            continue
        if ado and name.startswith("deep_output."):
            continue
        if not attention and (name.startswith("attention.") or name.startswith("f_beta.")):
            continue
        names.append(name)
    return names


def train_step(p, img_features, captions, *, tf, ado, attention, bert=False,
               alpha_c=1.0, lr=1e-4, dropout_masks=None, training=True, adam_state=None):
    """train.py:128-164 for one batch (encoder output given).  Returns
    (loss, grads dict, new params dict, preds, alphas)."""
    V, E = p["embedding.weight"].shape
    D = img_features.shape[2]
    names = trainable_names(V, D, E, ado, attention, bert)
    q = {k: v.clone().detach().requires_grad_(k in names) for k, v in p.items()}
    preds, alphas, _ = decoder_forward(q, img_features, captions, tf=tf, ado=ado, attention=attention,
                                       bert=bert, training=training, dropout_masks=dropout_masks)
    loss = caption_loss(preds, alphas, captions, alpha_c)
    loss.backward()
    grads = {k: q[k].grad.detach().clone() for k in names if q[k].grad is not None}
    newp = {k: v.detach().clone() for k, v in q.items()}
    adam_step(newp, grads, adam_state if adam_state is not None else {}, lr)
    return loss.detach(), grads, newp, preds.detach(), alphas.detach()


# ----------------------------------------------------------------------------
# Encoder trunks (encoder.py + torchvision 0.16 vgg19 / resnet152 restated)
# ----------------------------------------------------------------------------

VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]
RESNET152_LAYERS = [3, 8, 36, 3]


def vgg19_layer_list():
    """torchvision vgg19 cfg 'E' ``features`` with the final MaxPool dropped
    (encoder.py:24-27).  Items: ('conv', cin, cout, idx) | ('relu', idx) | ('pool', idx)."""
    out, cin, idx = [], 3, 0
    for v in VGG19_CFG:
        if v == "M":
            out.append(("pool", idx)); idx += 1
        else:
            out.append(("conv", cin, v, idx)); idx += 1
            out.append(("relu", idx)); idx += 1
            cin = v
    return out[:-1]


def make_vgg19_params(seed, scale=1.0):
    """Kaiming-normal (fan_out, relu) conv weights as torchvision initialises
    them, zero biases replaced by small uniform ones so the bias path is
    exercised.  Keys follow Encoder.state_dict(): ``net.<idx>.weight``."""
    rng = np.random.default_rng(seed)
    p = {}
    for item in vgg19_layer_list():
        if item[0] != "conv":
            continue
        _, cin, cout, idx = item
        std = scale * math.sqrt(2.0 / (cout * 9))
        p[f"net.{idx}.weight"] = torch.from_numpy((rng.standard_normal((cout, cin, 3, 3)) * std).astype(np.float32))
        p[f"net.{idx}.bias"] = torch.from_numpy(rng.uniform(-0.05, 0.05, cout).astype(np.float32))
    return p


def vgg19_forward(p, x):
    """encoder.py:33-40 with the VGG19 trunk: [B,3,H,W] -> [B, H/16*W/16, 512]."""
    for item in vgg19_layer_list():
        if item[0] == "conv":
            idx = item[3]
            x = F.conv2d(x, p[f"net.{idx}.weight"], p[f"net.{idx}.bias"], padding=1)
        elif item[0] == "relu":
            x = torch.relu(x)
        else:
            x = F.max_pool2d(x, 2, 2)
    x = x.permute(0, 2, 3, 1)
    return x.reshape(x.size(0), -1, x.size(-1))


def resnet152_blocks():
    """(prefix, inplanes, planes, stride, has_downsample) for every Bottleneck
    of torchvision resnet152 (expansion 4, stride on the 3x3 conv, v1.5)."""
    blocks, inplanes = [], 64
    for li, (n, planes) in enumerate(zip(RESNET152_LAYERS, [64, 128, 256, 512])):
        stride = 1 if li == 0 else 2
        for bi in range(n):
            s = stride if bi == 0 else 1
            ds = bi == 0 and (s != 1 or inplanes != planes * 4)
            blocks.append((f"net.{4 + li}.{bi}", inplanes, planes, s, ds))
            inplanes = planes * 4
    return blocks


def _bn_params(rng, c, prefix, p, randomize):
    if randomize:
        p[prefix + ".weight"] = torch.from_numpy(rng.uniform(0.5, 1.0, c).astype(np.float32))
        p[prefix + ".bias"] = torch.from_numpy(rng.uniform(-0.1, 0.1, c).astype(np.float32))
        p[prefix + ".running_mean"] = torch.from_numpy(rng.uniform(-0.1, 0.1, c).astype(np.float32))
        p[prefix + ".running_var"] = torch.from_numpy(rng.uniform(0.5, 1.5, c).astype(np.float32))
    else:
        p[prefix + ".weight"] = torch.ones(c); p[prefix + ".bias"] = torch.zeros(c)
        p[prefix + ".running_mean"] = torch.zeros(c); p[prefix + ".running_var"] = torch.ones(c)
    p[prefix + ".num_batches_tracked"] = torch.tensor(0, dtype=torch.long)


def make_resnet152_params(seed, randomize_bn=True, scale=1.0):
    rng = np.random.default_rng(seed)
    p = {}

    def conv(name, cout, cin, k):
        std = scale * math.sqrt(2.0 / (cout * k * k))
        p[name] = torch.from_numpy((rng.standard_normal((cout, cin, k, k)) * std).astype(np.float32))

    conv("net.0.weight", 64, 3, 7)
    _bn_params(rng, 64, "net.1", p, randomize_bn)
    for prefix, inplanes, planes, stride, ds in resnet152_blocks():
        conv(prefix + ".conv1.weight", planes, inplanes, 1); _bn_params(rng, planes, prefix + ".bn1", p, randomize_bn)
        conv(prefix + ".conv2.weight", planes, planes, 3); _bn_params(rng, planes, prefix + ".bn2", p, randomize_bn)
        conv(prefix + ".conv3.weight", planes * 4, planes, 1)
        # damp the last BN of each residual branch so 50 stacked blocks stay O(1)
        _bn_params(rng, planes * 4, prefix + ".bn3", p, randomize_bn)
        if randomize_bn:
            p[prefix + ".bn3.weight"] = p[prefix + ".bn3.weight"] * 0.2
        if ds:
            conv(prefix + ".downsample.0.weight", planes * 4, inplanes, 1)
            _bn_params(rng, planes * 4, prefix + ".downsample.1", p, randomize_bn)
    return p


def _bn(x, p, prefix, eps=1e-5):
    return F.batch_norm(x, p[prefix + ".running_mean"], p[prefix + ".running_var"],
                        p[prefix + ".weight"], p[prefix + ".bias"], training=False, eps=eps)


def resnet152_forward(p, x):
    """encoder.py:13-17,33-40: conv1/bn1/relu/maxpool + layer1..4 (BN in eval
    mode, train.py:122) -> [B, H/32*W/32, 2048]."""
    x = torch.relu(_bn(F.conv2d(x, p["net.0.weight"], stride=2, padding=3), p, "net.1"))
    x = F.max_pool2d(x, 3, 2, 1)
    for prefix, inplanes, planes, stride, ds in resnet152_blocks():
        idn = x
        out = torch.relu(_bn(F.conv2d(x, p[prefix + ".conv1.weight"]), p, prefix + ".bn1"))
        out = torch.relu(_bn(F.conv2d(out, p[prefix + ".conv2.weight"], stride=stride, padding=1), p, prefix + ".bn2"))
        out = _bn(F.conv2d(out, p[prefix + ".conv3.weight"]), p, prefix + ".bn3")
        if ds:
            idn = _bn(F.conv2d(x, p[prefix + ".downsample.0.weight"], stride=stride), p, prefix + ".downsample.1")
        x = torch.relu(out + idn)
    x = x.permute(0, 2, 3, 1)
    return x.reshape(x.size(0), -1, x.size(-1))


# ----------------------------------------------------------------------------
# BLEU (nltk 3.8.1 corpus_bleu restated; call sites train.py:330-333)
# ----------------------------------------------------------------------------

def _ngrams(seq, n):
    return [tuple(seq[i:i + n]) for i in range(len(seq) - n + 1)]


def _modified_precision(references, hypothesis, n):
    counts = Counter(_ngrams(hypothesis, n))
    max_counts = {}
    for ref in references:
        rc = Counter(_ngrams(ref, n))
        for ng in counts:
            max_counts[ng] = max(max_counts.get(ng, 0), rc[ng])
    clipped = sum(min(c, max_counts[ng]) for ng, c in counts.items())
    return clipped, max(1, sum(counts.values()))


def _closest_ref_length(references, hyp_len):
    return min((len(r) for r in references), key=lambda rl: (abs(rl - hyp_len), rl))


def corpus_bleu(list_of_references, hypotheses, weights=(0.25, 0.25, 0.25, 0.25)):
    """nltk.translate.bleu_score.corpus_bleu, nltk 3.8.1, default
    SmoothingFunction().method0, auto_reweigh=False."""
    num = Counter(); den = Counter()
    hyp_lengths = ref_lengths = 0
    for refs, hyp in zip(list_of_references, hypotheses):
        for i in range(1, len(weights) + 1):
            a, b = _modified_precision(refs, hyp, i)
            num[i] += a; den[i] += b
        hl = len(hyp)
        hyp_lengths += hl
        ref_lengths += _closest_ref_length(refs, hl)
    # brevity_penalty(closest_ref_len, hyp_len)
    if hyp_lengths > ref_lengths:
        bp = 1.0
    elif hyp_lengths == 0:
        bp = 0.0
    else:
        bp = math.exp(1 - ref_lengths / hyp_lengths)
    p_n = [Fraction(num[i], den[i], _normalize=False) for i in range(1, len(weights) + 1)]
    if num[1] == 0:
        return 0
    # method0: a zero precision becomes sys.float_info.min
    logs = []
    for w, p in zip(weights, p_n):
        if p.numerator != 0:
            logs.append(w * math.log(p))
        else:
            logs.append(w * math.log(sys.float_info.min))
    return bp * math.exp(math.fsum(logs))
