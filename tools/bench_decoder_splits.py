"""A/B the split-K counts of the per-step bf16 decoder GEMMs (SatPolicy.decoder_splits, per call) on the bench
workload (B=128, L=49, D=2048, E=512, V=10000, T=27, tf+ado+attention): decoder fwd + loss + bwd
timed with events, configurations interleaved over rounds in one process.

    SPLITS="0,0,0,0;2,0,0,0;..." python tools/bench_decoder_splits.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import sat_amd  # noqa: E402
from sat_amd.data import synthetic_captions  # noqa: E402

dev = torch.device("cuda")
B, L, D, V, T = 128, 49, 2048, 10000, 27
torch.manual_seed(0)
dec = sat_amd.Decoder(V, D, tf=True, ado=True, attention=True).to(dev).train()
feats = torch.randn(B, L, D, device=dev).bfloat16()
caps = synthetic_captions(B, T, V, generator=torch.Generator().manual_seed(1), device=dev)
CONFIGS = [tuple(int(v) for v in c.split(",")) for c in
           os.environ.get("SPLITS", "0,0,0,0;2,0,0,0;8,0,0,0;0,4,0,0;0,16,0,0;0,0,8,0;0,0,32,0;0,0,0,12;0,0,0,36").split(";")]


def step():
    preds, alphas = dec(feats, caps)
    loss, _ = sat_amd.caption_loss(preds, alphas, caps)
    loss.backward()


times = {c: [] for c in CONFIGS}
for rnd in range(4):
    for cfg in CONFIGS:
        dec.policy = sat_amd.Policy(decoder_splits=cfg)
        step()
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(3):
            step()
        en.record()
        en.synchronize()
        times[cfg].append(st.elapsed_time(en) / 3)
dec.policy = None
for cfg in CONFIGS:
    print(f"splits h,c,g,dh={cfg}: {statistics.median(times[cfg]):.3f} ms (min {min(times[cfg]):.3f})", flush=True)
