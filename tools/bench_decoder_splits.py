"""A/B the split-K counts of the per-step bf16 decoder GEMMs (SatPolicy.decoder_splits) and the transposed weight
copies (Decoder.transposed_weights) on the bench workload (L=49, D=2048, E=512, V=10000, T=27, tf+ado+attention),
one process: per configuration the per-step kernel groups (diagnostics.decoder_step_kernels, back to back) and the
decoder fwd + loss + bwd time (events, split target 64 as in the overlapped bench).

    CONFIGS="tr:h,c,g,dh[:attn_bwd_chunks];..." B=128 python tools/bench_decoder_splits.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import sat_amd  # noqa: E402
from sat_amd.data import synthetic_captions  # noqa: E402
from sat_amd.diagnostics import decoder_step_kernels  # noqa: E402

dev = torch.device("cuda")
B = int(os.environ.get("B", "128"))
L, D, V, T = 49, 2048, 10000, 27
torch.manual_seed(0)
dec = sat_amd.Decoder(V, D, tf=True, ado=True, attention=True).to(dev).train()
dec.split_target = 64
feats = torch.randn(B, L, D, device=dev).bfloat16()
caps = synthetic_captions(B, T, V, generator=torch.Generator().manual_seed(1), device=dev)
CONFIGS = []
for c in os.environ.get("CONFIGS", "0:0,0,0,0;1:0,0,0,0;1:0,0,0,0:1;1:0,0,0,0:2").split(";"):
    f = c.split(":") + ["0"]
    CONFIGS.append((int(f[0]), tuple(int(v) for v in f[1].split(",")), int(f[2])))


def step():
    preds, alphas = dec(feats, caps)
    loss, _ = sat_amd.caption_loss(preds, alphas, caps)
    loss.backward()


def configure(cfg):
    dec.transposed_weights = bool(cfg[0])
    dec._lp_versions = None   # re-cast the shadow (and refresh the transposed copies when on)
    dec.policy = sat_amd.Policy(decoder_splits=cfg[1], attn_bwd_chunks=cfg[2])


times = {c: [] for c in CONFIGS}
groups = {}
for rnd in range(3):
    for cfg in CONFIGS:
        configure(cfg)
        step()
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(3):
            step()
        en.record()
        en.synchronize()
        times[cfg].append(st.elapsed_time(en) / 3)
        if rnd == 0:
            groups[cfg] = decoder_step_kernels(dec, feats, caps, reps=20)[0]
for cfg in CONFIGS:
    g = groups[cfg]
    print(f"transposed={cfg[0]} splits h,c,g,dh={cfg[1]} bwd_chunks={cfg[2]}: fwd+bwd {statistics.median(times[cfg]):.3f} ms; per step "
          f"{sum(g.values()):.1f} us: " + " ".join(f"{k} {v:.2f}" for k, v in g.items()), flush=True)
