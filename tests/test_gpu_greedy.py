"""The fused greedy decoder step and the deterministic embedding gradient (round 6).

* Fused greedy step (SatPolicy.greedy_step = 0, bf16, teacher forcing off: decoder.py:118-133 per step): the embedding
  half of the LSTM input GEMM from a token table built once per forward, dropout drawn inside the LSTM kernel, the ado
  head's f_z beside the context GEMM, f_h + ReLUs + combine in one launch, the vocabulary head writing per-block argmax
  partials.  Checked against the bf16 rounding mirror of the oracle (oracle/sat_oracle.py bf16_mirror, fp64)
  conditioned on the tokens the HIP decoder fed itself (decoder.py:131-133: the argmax feedback is a constant for
  autograd), with the seeded dropout masks rebuilt on the host from the decoder's seed -- so the in-kernel mask draw
  of both forms is pinned too.
* Dense embedding gradient (SatPolicy.embed_grad = 0): per-token sums in row order (one sort launch, piece sums, a
  fix-up for tokens whose rows span pieces), bit-identical across runs, against the fp32-atomic form and the oracle.

Reference: decoder.py:87,107-133,149-158 (embedding, LSTM input, head, greedy feedback), train.py:150-164.
"""
import numpy as np
import pytest
import torch

from oracle import sat_oracle as O
import test_gpu_shapes as S

pytestmark = pytest.mark.gpu
DEV = "cuda"
M64 = (1 << 64) - 1


@pytest.fixture(scope="module")
def sat():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import sat_amd
    return sat_amd


def _mix32(x):
    x = x ^ (x >> np.uint64(33))
    x = x * np.uint64(0xff51afd7ed558ccd)
    x = x ^ (x >> np.uint64(33))
    x = x * np.uint64(0xc4ceb9fe1a85ec53)
    x = x ^ (x >> np.uint64(33))
    return x & np.uint64(0xffffffff)


def host_dropout_masks(seed, B, T1, E):
    """The keep-mask the kernels draw for a forward whose device seed counter is 0 (lstm.hip dropout_keep): [T1, B, E]
    as the oracle takes it."""
    b = np.arange(B, dtype=np.uint64)[None, :, None]
    t = np.arange(T1, dtype=np.uint64)[:, None, None]
    e = np.arange(E, dtype=np.uint64)[None, None, :]
    with np.errstate(over="ignore"):
        x = np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15) + ((b << np.uint64(40)) ^ (t << np.uint64(20)) ^ e)
        keep = _mix32(x) & np.uint64(1)
    return torch.from_numpy(keep.astype(np.float32))


def _greedy_seeded(sat, c, form):
    """A bf16 greedy train-mode forward + backward with dropout drawn from the decoder's seed (no injected mask)."""
    torch.manual_seed(1234)   # the decoder's dropout seed is drawn from torch's generator: one draw for every process
    dec = S._decoder(sat, c).train()
    dec.policy = sat.Policy(greedy_step=form)
    caps = c["caps"].to(DEV)
    feats = c["feats"].to(DEV).bfloat16()
    preds, alphas = dec(feats, caps)
    pad, skip = sat.special_ids(c["bert"])
    loss, _ = sat.caption_loss(preds, alphas, caps, 1.0, pad, skip)
    loss.backward()
    torch.cuda.synchronize()
    params = dict(dec.named_parameters())
    grads = {n: params[n].grad.detach().float().cpu().clone() for n in dec.active_param_names()}
    return dec, dict(loss=loss.item(), preds=preds.detach().float().cpu(), alphas=alphas.detach().float().cpu(),
                     grads=grads, tokens=dec.last_tokens.long().cpu())


# bounds against the bf16 rounding mirror of the oracle (oracle/sat_oracle.py bf16_mirror, fp64) at these B <= 4, T = 6-8
# cases: measured <= 2.4e-3 per parameter (profiles/r6_s3/py_1_debug_greedy.log: both forms, seeded and injected masks,
# with and without the ado head); against the plain fp32 oracle the same steps differ by up to 0.2 for some seeds
# (bf16 rounding of the ReLU'd logits near zero), which is why the mirror is the reference here.  The step is
# bit-reproducible run to run, but with dropout drawn from the decoder's seed the error depends on the
# draw: where a draw flips a bf16 rounding of a per-step operand the head and LSTM gradients move by up to 2.9e-2
# ([True-1], profiles/r6_s70: torch's default generator is seeded per process here, so each process drew other
# masks; profiles/r6_s71: 1 of 3 processes) -- hence 3e-2, and _greedy_seeded now fixes the draw
MIRROR_TOL = 3e-2


def _mirror_fed(c, tokens):
    with O.bf16_mirror():
        return S._oracle_fed(c, tokens, torch.float64)


def _assert_mirror(h, o, tol=MIRROR_TOL):
    loss_m, g_m, _, preds_m, alphas_m = o
    assert S.rel(h["preds"], preds_m) < 1e-2
    assert S.rel(h["alphas"], alphas_m) < 1e-2
    assert abs(h["loss"] - loss_m.item()) <= 1e-3 * abs(loss_m.item())
    assert sorted(h["grads"]) == sorted(g_m)
    errs = S._grad_errors(h, {n: g.float() for n, g in g_m.items()})
    print("bf16 gradient errors vs the fed-token bf16 mirror:", {n: round(e, 5) for n, e in errs.items()})
    bad = {n: e for n, e in errs.items() if e >= tol}
    assert not bad, bad


@pytest.mark.parametrize("form", [0, 1])
@pytest.mark.parametrize("ado", [True, False])
def test_greedy_step_seeded_dropout_matches_oracle(sat, form, ado):
    """Both greedy forms (0 = fused, 1 = per-op) in training mode with seeded dropout: the masks rebuilt on the host
    from the seed, the fed-token bf16 mirror oracle."""
    D, Lf, E, V, T = 512, 196, 512, 2600, 8
    c = S._make_case(D, Lf, E, V, T, False, ado, False, 4, 23)
    dec, h = _greedy_seeded(sat, c, form)
    c = dict(c, masks=host_dropout_masks(dec._seed_host, 4, T - 1, E))
    _assert_mirror(h, _mirror_fed(c, h["tokens"]))


def test_greedy_fused_tokens_are_argmax_of_preds(sat):
    """The fused head's argmax partials and the final reduction feed back exactly torch.argmax of the stored bf16 logits
    (first index on ties, decoder.py:132), at the bench's greedy shape (B = 64, V = 10000: 313 column blocks)."""
    c = S._bench_case("b64_greedy_st64")
    h = S._hip_step(sat, c, torch.bfloat16, split_target=c["split_target"])
    ids = h["preds"].argmax(2)
    assert torch.equal(h["tokens"][:, 1:], ids[:, :-1])
    assert torch.equal(h["tokens"][:, 0], torch.zeros_like(h["tokens"][:, 0]))


def test_greedy_fused_odd_vocabulary_and_small_batch(sat):
    """A vocabulary that is not a multiple of the 32-column block (nor of 4: the head's scalar store path) and a batch
    of 3 rows: the fused head against the fed-token oracle, and the fed tokens = argmax of the stored logits."""
    D, Lf, E, V, T = 512, 49, 512, 1003, 6
    c = S._make_case(D, Lf, E, V, T, False, True, False, 3, 29)
    h = S._hip_step(sat, c, torch.bfloat16)
    assert torch.equal(h["tokens"][:, 1:], h["preds"].argmax(2)[:, :-1])
    _assert_mirror(h, _mirror_fed(c, h["tokens"]))


def _pad_heavy_case(Bn, T, seed):
    """Captions that are mostly <pad>: the fed token 3 repeats over nearly every row, so its segment of the sorted rows
    spans many 32-row pieces (the fix-up path), next to short segments of rare tokens."""
    c = S._make_case(2048, 49, 512, 10000, T, True, True, False, Bn, seed)
    caps = c["caps"].clone()
    caps[:, 3:] = 3
    caps[0, 3:6] = torch.tensor([17, 17, 9999])
    c["caps"] = caps
    return c


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_embedding_gradient_sorted_matches_atomic(sat, dtype):
    c = _pad_heavy_case(8, 27, 41)
    a = S._hip_step(sat, c, dtype, policy=sat.Policy(embed_grad=0))
    b = S._hip_step(sat, c, dtype, policy=sat.Policy(embed_grad=1))
    ga, gb = a["grads"]["embedding.weight"], b["grads"]["embedding.weight"]
    assert ((ga - gb).norm() / gb.norm()).item() < 1e-6
    assert torch.equal(ga != 0, gb != 0)   # exactly the fed tokens' rows are touched
    if dtype == torch.float32:
        o = S._oracle(c, torch.float32)
        ref = o[1]["embedding.weight"]
        assert ((ga - ref).norm() / ref.norm()).item() < 2e-4


def test_embedding_gradient_sorted_bit_identical(sat):
    c = _pad_heavy_case(8, 27, 43)
    runs = [S._hip_step(sat, c, torch.bfloat16)["grads"]["embedding.weight"] for _ in range(3)]
    for r in runs[1:]:
        assert torch.equal(r, runs[0])
