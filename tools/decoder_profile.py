"""Decoder train step alone (bench shape: B=128, ResNet152 features L=49 x D=2048, V=10000, T=27,
bf16, hipGraph replay): wall time per step vs the sum of its kernels' durations, from a rocprofv3
kernel trace of this script.
    rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python tools/decoder_profile.py
    python tools/decoder_profile.py --analyze DIR/run_kernel_trace.csv"""
import csv
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def analyze(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the timed replays are bracketed by the marker kernels of the last 10 replays: take the last 10 steps
    marks = [i for i, r in enumerate(rows) if "tokens_kernel" in r["Kernel_Name"]]   # first kernel of a forward
    if len(marks) < 11:
        raise SystemExit(f"need >= 11 decoder steps in the trace, found {len(marks)}")
    seg = rows[marks[-11]:marks[-1]]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(rows[marks[-1]]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    by = {}
    for r in seg:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")[:60]
        d = by.setdefault(k, [0, 0])
        d[0] += 1
        d[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    steps = 10
    print(f"wall {((t1 - t0) / steps) / 1e3:.1f} us/step, kernels {busy / steps / 1e3:.1f} us/step, "
          f"{len(seg) / steps:.0f} launches/step, gap {((t1 - t0) - busy) / steps / 1e3:.1f} us/step")
    for k, (n, ns) in sorted(by.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f"  {k:60s} {n / steps:6.1f}/step {ns / steps / 1e3:9.1f} us/step  avg {ns / n / 1e3:7.2f} us")


def main():
    import torch
    import sat_amd
    from sat_amd.data import synthetic_captions
    dev = "cuda"
    torch.manual_seed(0)
    B, L, D, V, T = 128, 49, 2048, 10000, 27
    dec = sat_amd.Decoder(V, D, tf=True, ado=True, attention=True).to(dev).train()
    opt = sat_amd.Adam(dec.parameters(), lr=1e-4)
    g = torch.Generator().manual_seed(1)
    feats = (torch.randn(B, L, D, generator=g).relu()).bfloat16().to(dev)
    caps = synthetic_captions(B, T, V, generator=g, device=dev)
    pad_id, skip_ids = sat_amd.special_ids(False)

    def step():
        preds, alphas = dec(feats, caps)
        loss, _ = sat_amd.caption_loss(preds, alphas, caps, pad_id=pad_id, skip_ids=skip_ids)
        loss.backward()
        return loss
    for _ in range(3):
        opt.zero_grad()
        step()
        opt.step()
    torch.cuda.synchronize()
    opt.zero_grad(set_to_none=True)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        step()
    for _ in range(3):
        gr.replay()
        opt.step()
    torch.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        gr.replay()
        opt.step()
    torch.cuda.synchronize()
    print(f"decoder step (graph fwd+loss+bwd + eager Adam): {(time.perf_counter() - t0) / n * 1e3:.3f} ms")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        main()
