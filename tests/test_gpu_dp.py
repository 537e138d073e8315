"""Data parallelism on the HIP kernels (the reference is single-device, train.py:163-164).

Two fresh rank processes (tests/dp_rank_worker.py, gloo, both on cuda:0) each run their half of a
global fp32 batch through the HIP decoder, with the bucketed gradient all-reduce of
sat_amd.distributed in both forms bench.py / train.py use (eager phase hooks; two captured
hipGraphs with the async bucket all-reduce between the replays), then the fused Adam step.  The
averaged gradients and post-Adam weights must equal a single-process full-batch HIP run (both loss
terms are means over equal-size local sets), and the library-drawn dropout masks must differ
between ranks (decoder.py:121-125 draws an independent mask per sample).
"""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def sat():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import sat_amd
    return sat_amd


def _full_batch(sat, case):
    sys.path.insert(0, HERE)
    import dp_rank_worker as W
    c = W.DP_CASES[case]
    p, feats, caps, mask = W.case_inputs(c)
    dec = W.make_decoder(sat, p, torch.device("cuda"), c)
    dec.dropout_mask = mask
    opt = sat.Adam(dec.parameters(), lr=c["lr"])
    opt.zero_grad()
    caps_d = caps.cuda()
    preds, alphas = dec(feats.cuda(), caps_d)
    sat.caption_loss(preds, alphas, caps_d)[0].backward()
    torch.cuda.synchronize()
    grads = W.snapshot(dec)
    opt.step()
    torch.cuda.synchronize()
    return grads, W.weights(dec)


# toy fp32 (the exact-parity path) and cfg3's per-rank shape in bf16 (ResNet152 / COCO decoder, 64 images per rank,
# bench.py's split target for B <= 64): in bf16 every per-row product of the two half batches is the full batch's
# bit for bit up to the exact factor 2 of the loss mean, so the averaged gradients differ from the full batch's only
# by the fp32 summation order of the batched weight-gradient GEMMs and the embedding scatter-add
# (gradient norm, gradient element / max, weights compared where |g| > this share of max|g|): in bf16 the two batch
# sizes take different split-K paths in the head's batched products, whose fp32 rounding differences then move bf16
# roundings downstream; a gradient element near zero can change sign, and Adam's first step moves it by lr * sign
TOL = {"toy_fp32": (5e-4, 2e-3, 1e-4), "cfg3_bf16": (2e-3, 2e-2, 5e-2)}


@pytest.mark.parametrize("case", ["toy_fp32", "cfg3_bf16"])
def test_dp_two_ranks_equal_full_batch(sat, tmp_path, case):
    world = 2
    init = tmp_path / "init"
    outs = [tmp_path / f"rank{r}.pt" for r in range(world)]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dp_rank_worker.py"), str(r), str(world),
                               str(init), str(outs[r]), case], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(world)]
    logs = []
    for pr in procs:
        try:
            logs.append(pr.communicate(timeout=240)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for pr, log in zip(procs, logs):
        assert pr.returncode == 0, log[-3000:]
    res = [torch.load(o, weights_only=True) for o in outs]
    g_full, w_full = _full_batch(sat, case)
    lr = 1e-4
    tol_norm, tol_elem, sure_share = TOL[case]
    for form in ("eager", "graph"):
        for r in range(world):
            g, w = res[r][f"{form}_grads"], res[r][f"{form}_weights"]
            assert sorted(g) == sorted(g_full)
            for n, ref in g_full.items():
                got = g[n]
                assert torch.isfinite(got).all(), (form, r, n)
                scale = ref.abs().max().item()
                if ref.norm().item() < 1e-7:   # attention.v.bias: analytically zero
                    assert got.abs().max().item() < 1e-5, (form, n)
                    continue
                # mean of the two half-batch gradients == full-batch gradient, up to fp32 summation order
                assert ((got - ref).norm() / ref.norm()).item() < tol_norm, (form, r, n)
                assert (got - ref).abs().max().item() <= tol_elem * scale, (form, r, n)
                # Adam's first step moves every weight by ~lr * sign(g): compare where the sign is not
                # at the fp32 noise level
                sure = ref.abs() > sure_share * scale
                dw = (w[n] - w_full[n]).abs()
                assert dw[sure].max().item() <= 2e-3 * lr + 1e-6, (form, r, n)
        # both ranks hold identical averaged gradients and weights (replicated optimiser)
        for n in g_full:
            assert torch.equal(res[0][f"{form}_grads"][n], res[1][f"{form}_grads"][n]), (form, n)
            assert torch.equal(res[0][f"{form}_weights"][n], res[1][f"{form}_weights"][n]), (form, n)
    # library-drawn dropout: independent per rank in train mode, identical in eval mode
    assert torch.equal(res[0]["eval_preds"], res[1]["eval_preds"])
    assert not torch.equal(res[0]["train_preds"], res[1]["train_preds"])


def test_dp_rccl_single_rank_equals_full_batch(sat, tmp_path):
    """The RCCL leg of the same schedule (bench.py's default backend): one rank over the nccl backend (RCCL) on the
    one GPU of the box, so torch.distributed's RCCL communicator, the ReduceOp.AVG bucket all-reduce of
    sat_amd.distributed (eager hooks and the async form between the two graph replays) and their stream ordering run
    on the device; with one rank the average is the identity, so both forms must reproduce the full-batch run."""
    init, out = tmp_path / "init", tmp_path / "rank0.pt"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", SAT_DP_BACKEND="nccl")
    pr = subprocess.run([sys.executable, os.path.join(HERE, "dp_rank_worker.py"), "0", "1", str(init), str(out),
                         "toy_fp32"], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=240)
    assert pr.returncode == 0, pr.stdout[-3000:]
    res = torch.load(out, weights_only=True)
    assert res["backend"] == "nccl" and res["rccl_version"], res.get("backend")
    g_full, w_full = _full_batch(sat, "toy_fp32")
    tol_norm, tol_elem, _ = TOL["toy_fp32"]
    for form in ("eager", "graph"):
        g, w = res[f"{form}_grads"], res[f"{form}_weights"]
        assert sorted(g) == sorted(g_full)
        for n, ref in g_full.items():
            got = g[n]
            assert torch.isfinite(got).all(), (form, n)
            if ref.norm().item() < 1e-7:   # attention.v.bias: analytically zero
                assert got.abs().max().item() < 1e-5, (form, n)
                continue
            assert ((got - ref).norm() / ref.norm()).item() < tol_norm, (form, n)
            assert (got - ref).abs().max().item() <= tol_elem * ref.abs().max().item(), (form, n)
            assert torch.isfinite(w[n]).all(), (form, n)
