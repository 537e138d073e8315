"""Trunk forward as one B=128 hipGraph vs S concurrent graphs of B/S images on S streams
(kernels of the streams interleave: one stream's prologue / tail / under-filled launch beside
another's main loop).  Prints ms per 128 images for each split.
    python tools/split_ab.py [network] [splits...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import sat_amd  # noqa: E402

net = sys.argv[1] if len(sys.argv) > 1 else "resnet152"
splits = [int(s) for s in sys.argv[2:]] or [1, 2, 4]
B = 128
torch.manual_seed(0)
enc = sat_amd.Encoder(net, dtype=torch.bfloat16).cuda().eval()
imgs = torch.randn(B, 3, 224, 224, device="cuda")
res = {}
for S in splits:
    b = B // S
    streams = [torch.cuda.Stream() for _ in range(S)]
    graphs, outs = [], []
    for k in range(S):
        x = imgs[k * b:(k + 1) * b].contiguous()
        with torch.no_grad():
            enc(x)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            with torch.no_grad():
                outs.append(enc(x))
        graphs.append(g)
    torch.cuda.synchronize()
    main = torch.cuda.current_stream()

    def once():
        ev = torch.cuda.Event()
        ev.record(main)
        for s, g in zip(streams, graphs):
            s.wait_event(ev)
            with torch.cuda.stream(s):
                g.replay()
        for s in streams:
            main.wait_stream(s)

    for _ in range(3):
        once()
    torch.cuda.synchronize()
    best = []
    for rep in range(3):
        n = 20
        t0 = time.perf_counter()
        for _ in range(n):
            once()
        torch.cuda.synchronize()
        best.append((time.perf_counter() - t0) / n * 1e3)
    full = torch.cat(outs, 0)
    res[S] = (min(best), full)
    print(f"split {S}: {min(best):.3f} ms per {B} images  (reps {', '.join(f'{x:.3f}' for x in best)})", flush=True)
    del graphs
ref = res[splits[0]][1].float()
for S in splits[1:]:
    d = (res[S][1].float() - ref).abs().max().item()
    print(f"split {S} vs {splits[0]}: max |diff| {d:.3e}")
