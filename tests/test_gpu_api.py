"""Public-API behaviour of the modules around the HIP path (train.py:133-164 call pattern).

* caption_loss returns a loss the caller may scale out of place or in place before backward (gradient
  accumulation divides the loss, AMP-style loops scale it in place) with the gradient scaled accordingly;
* a decoder forward keeps its own copy of the SatPolicy it ran with: editing dec.policy between a forward and its
  (deferred) backward changes nothing, because the workspace regions are placed from the forward's policy.
"""
import numpy as np
import pytest
import torch

from oracle import sat_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def sat():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import sat_amd
    return sat_amd


def _setup(sat, seed=5):
    V, D, Lf, E, B, T = 60, 64, 16, 512, 3, 7
    p = O.make_decoder_params(V, D, E, True, seed)
    rng = np.random.default_rng(seed)
    feats = torch.from_numpy(rng.standard_normal((B, Lf, D)).astype(np.float32)).to(DEV)
    caps = O.make_captions(B, T, V, seed + 1).to(DEV)
    dec = sat.Decoder(V, D, tf=True, ado=True, attention=True)
    dec.load_state_dict(p, strict=True)
    return dec.to(DEV).eval(), feats, caps


def _grads(dec):
    return {n: p.grad.detach().clone() for n, p in dec.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("scale_mode", ["div", "inplace"])
def test_loss_can_be_scaled_before_backward(sat, scale_mode):
    dec, feats, caps = _setup(sat)
    preds, alphas = dec(feats, caps)
    loss, _ = sat.caption_loss(preds, alphas, caps)
    loss.backward()
    torch.cuda.synchronize()
    ref = _grads(dec)
    dec.zero_grad(set_to_none=True)
    preds, alphas = dec(feats, caps)
    loss, _ = sat.caption_loss(preds, alphas, caps)
    if scale_mode == "div":
        loss = loss / 2
    else:
        loss.mul_(0.5)
    loss.backward()
    torch.cuda.synchronize()
    got = _grads(dec)
    assert sorted(got) == sorted(ref)
    for n, g in got.items():
        # the dense embedding gradient is a scatter-add with fp32 atomics (summation order varies run to run)
        tol = 1e-6 * ref[n].abs().max().item() if n == "embedding.weight" else 1e-12
        assert torch.allclose(g, ref[n] * 0.5, rtol=1e-6, atol=tol), n


def test_policy_edit_between_forward_and_deferred_backward(sat):
    dec, feats, caps = _setup(sat)
    feats = feats.bfloat16()
    dec.train()
    dec.dropout_mask = torch.ones(feats.shape[0], caps.shape[1] - 1, 512, dtype=torch.uint8, device=DEV)

    def step(edit):
        dec.zero_grad(set_to_none=True)
        dec.policy = sat.Policy(decoder_splits=[2, 2, 2, 2])
        dec.defer_recurrent_backward(True)
        preds, alphas = dec(feats, caps)
        sat.caption_loss(preds, alphas, caps)[0].backward()
        if edit:   # a different split layout after the forward: the deferred phase 2 must not see it
            dec.policy.decoder_splits[:] = [4, 4, 4, 4]
            dec.policy.attn_bwd_chunks = 3
        dec.finish_backward()
        dec.defer_recurrent_backward(False)
        torch.cuda.synchronize()
        return _grads(dec)
    a, b = step(False), step(True)
    # a backward that read the edited policy would place the workspace regions at other offsets (garbage gradients,
    # O(1) off); the forward's own copy keeps phase 2 on the forward's layout, and the step is bit-reproducible (no
    # per-step product takes the atomic split-K: csrc/decoder.hip ragged_splits), so the two backwards agree exactly
    for n in a:
        assert torch.equal(a[n], b[n]), (n, ((a[n] - b[n]).abs().max() / a[n].abs().max()).item())


@pytest.mark.parametrize("splits", [None, [1, 1, 1, 1], [2, 2, 2, 2]])
def test_small_batch_training_step_bit_reproducible(sat, splits):
    """Three identical bf16 training steps at B = 3, T = 7, D = 64 (K = 5E + D = 2624 for the recurrent dh product:
    41 k-tiles, no whole divisor fits -- before ragged_splits it ran on fp32 atomics and the gradients differed run
    to run, profiles/r6_s54) give bit-identical gradients, every parameter including the dense embedding's."""
    dec, feats, caps = _setup(sat)
    feats = feats.bfloat16()
    dec.train()
    dec.dropout_mask = torch.ones(feats.shape[0], caps.shape[1] - 1, 512, dtype=torch.uint8, device=DEV)
    if splits is not None:
        dec.policy = sat.Policy(decoder_splits=splits)

    def step():
        dec.zero_grad(set_to_none=True)
        preds, alphas = dec(feats, caps)
        sat.caption_loss(preds, alphas, caps)[0].backward()
        torch.cuda.synchronize()
        return _grads(dec)
    ref = step()
    for _ in range(2):
        got = step()
        for n in ref:
            assert torch.equal(ref[n], got[n]), (n, ((ref[n] - got[n]).abs().max() / ref[n].abs().max()).item())
