"""Diagnostics: test_gpu_api.py::test_policy_edit_between_forward_and_deferred_backward's two steps repeated in one
process; prints, per repeat, the largest relative gradient difference between the plain and the edited-policy step
and between two plain steps (run-to-run), so a nondeterministic reduction shows up as a nonzero second column."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402

import sat_amd as sat  # noqa: E402
import test_gpu_api as A  # noqa: E402

dec, feats, caps = A._setup(sat)
feats = feats.bfloat16()
dec.train()
dec.dropout_mask = torch.ones(feats.shape[0], caps.shape[1] - 1, 512, dtype=torch.uint8, device="cuda")


# SAT_WS_FILL=zero|rand: every torch.empty inside decoder.py (the workspace, preds, alphas) zeroed / filled with
# fresh random bytes, to tell a read of uninitialised workspace apart from a nondeterministic reduction
FILL = os.environ.get("SAT_WS_FILL", "")
if FILL:
    _dmod = sys.modules[type(dec).__module__]
    _empty = torch.empty

    class _TorchFill:
        def __getattr__(self, k):
            return getattr(torch, k)

        def empty(self, *a, **k):
            t = _empty(*a, **k)
            if FILL == "zero":
                t.zero_()
            elif t.dtype == torch.uint8:
                t.random_(0, 256)
            return t
    _dmod.torch = _TorchFill()

EXTRA = dict(kv.split("=") for kv in sys.argv[2:])   # extra SatPolicy fields, e.g. attn_bwd_chunks=1
EXTRA = {k: int(v) for k, v in EXTRA.items()}
SPLITS = [int(x) for x in os.environ.get("SAT_SPLITS", "2,2,2,2").split(",")]   # Policy.decoder_splits


def step(edit):
    dec.zero_grad(set_to_none=True)
    dec.policy = sat.Policy(decoder_splits=SPLITS, **EXTRA)
    dec.defer_recurrent_backward(True)
    preds, alphas = dec(feats, caps)
    step.preds = preds.detach().float().clone()
    sat.caption_loss(preds, alphas, caps)[0].backward()
    step.phase1 = {n: p.grad.detach().clone() for n, p in dec.named_parameters() if p.grad is not None}
    step.b1 = dec.grad_bucket(1).detach().clone()
    ws = dec._pending_bwd[4] if dec._pending_bwd is not None else None
    step.ws1 = ws.clone() if ws is not None else None   # the workspace after phase 1
    if edit:
        dec.policy.decoder_splits[:] = [4, 4, 4, 4]
        dec.policy.attn_bwd_chunks = 3
    dec.finish_backward()
    dec.defer_recurrent_backward(False)
    torch.cuda.synchronize()
    step.ws2 = ws.clone() if ws is not None else None   # ... and after phase 2
    return A._grads(dec)


def ws_diff(a, b, gap=1024):
    """Byte ranges (clusters of differing 4-byte words, split at gaps > gap bytes) where two workspaces differ."""
    if a is None or b is None or a.numel() != b.numel():
        return "n/a"
    n = a.numel() // 4 * 4
    idx = torch.nonzero(a[:n].view(torch.int32) != b[:n].view(torch.int32)).flatten().cpu().tolist()
    out, s0, prev = [], None, None
    for i in idx:
        if s0 is None:
            s0 = prev = i
        elif (i - prev) * 4 > gap:
            out.append((s0 * 4, prev * 4 + 4))
            s0 = i
        prev = i
    if s0 is not None:
        out.append((s0 * 4, prev * 4 + 4))
    return out[:12]


def worst(a, b):
    out = {}
    for n in a:
        d = (a[n] - b[n]).abs().max().item()
        if d:
            out[n] = d / max(a[n].abs().max().item(), 1e-30)
    return out


ref = step(False)
ref_preds, ref_p1, ref_b1 = step.preds, step.phase1, step.b1
ref_ws1, ref_ws2 = step.ws1, step.ws2
if ref_ws2 is not None:
    print("workspace bytes", ref_ws2.numel(), flush=True)
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    p = step(False)
    dp = (step.preds - ref_preds).abs().max().item()
    w1 = worst(ref_p1, step.phase1)
    wp = worst(ref, p)
    top = sorted(wp.items(), key=lambda kv: -kv[1])[:4]
    db1 = (step.b1 - ref_b1).abs().max().item() / ref_b1.abs().max().item()
    print(i, f"preds {dp:.2e}", f"bucket1 after phase 1 {db1:.2e}", "phase1:", {k: f"{v:.1e}" for k, v in sorted(w1.items(), key=lambda kv: -kv[1])[:3]},
          "final:", {k: f"{v:.1e}" for k, v in top}, "n_differing", len(wp), flush=True)
    if os.environ.get("SAT_WS_DIFF"):
        print("   ws after phase 1 differs at", ws_diff(ref_ws1, step.ws1), flush=True)
        print("   ws after phase 2 differs at", ws_diff(ref_ws2, step.ws2), flush=True)
    if os.environ.get("SAT_DHG"):   # "offset,rows,cols": an fp32 region of the workspace, per-row difference figures
        off, rows, cols = (int(x) for x in os.environ["SAT_DHG"].split(","))
        ra = ref_ws2[off:off + rows * cols * 4].view(torch.float32).view(rows, cols)
        rb = step.ws2[off:off + rows * cols * 4].view(torch.float32).view(rows, cols)
        for r in range(rows):
            d = (ra[r] - rb[r]).abs()
            nz = int((d > 0).sum())
            if nz:
                k = int(d.argmax())
                print(f"   row {r}: {nz} differ, max {d[k].item():.3e} at col {k} (ref {ra[r, k].item():.6e}, "
                      f"got {rb[r, k].item():.6e}), row max {ra[r].abs().max().item():.3e}", flush=True)
