"""Fused bottleneck kernel (csrc/convblock.hip) vs the three conv launches it replaces, and the whole
ResNet152 trunk as one hipGraph with the fused blocks on / off.  B = 128, bf16.
    python tools/block_ab.py"""
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import sat_amd  # noqa: E402
from sat_amd import ops  # noqa: E402

B = 128
dev = "cuda"
g = torch.Generator().manual_seed(0)
x = torch.randn(B, 14, 14, 1024, generator=g).relu().bfloat16().to(dev)


def conv(cout, cin, k):
    w = (torch.randn(cout, k, k, cin, generator=g) * math.sqrt(2.0 / (k * k * cin))).bfloat16().to(dev)
    return w, (0.1 * torch.randn(cout, generator=g)).to(dev)


(w1, b1), (w2, b2), (w3, b3) = conv(256, 1024, 1), conv(256, 256, 3), conv(1024, 256, 1)
frags = [(ops.mfma_frag_layout(w.reshape(w.shape[0], -1)), b) for w, b in ((w1, b1), (w2, b2), (w3, b3))]
y = torch.empty_like(x)


def unfused():
    a = ops.conv2d_nhwc(x, w1, b1, 1, 0, True)
    c = ops.conv2d_nhwc(a, w2, b2, 1, 1, True)
    return ops.conv2d_nhwc(c, w3, b3, 1, 0, True, residual=x, out=y)


def fused():
    return ops.bottleneck_fused(x, *frags, out=y)


def timeit(f, n=50):
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            f()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / n * 1e3)
    return best


flops = 2 * B * 196 * (1024 * 256 + 9 * 256 * 256 + 256 * 1024)
for name, f in (("unfused", unfused), ("fused", fused), ("unfused", unfused), ("fused", fused)):
    us = timeit(f)
    print(f"block {name:8s} {us:8.2f} us  {flops / us / 1e6:7.1f} TFLOP/s  (frac {flops / us / 1e6 / 2500:.3f})",
          flush=True)
lib = sat_amd._lib.lib()
for pf, abl in ((2, 0), (2, 128), (2, 0), (2, 128)):
    assert lib.sat_bottleneck_set_experiment(pf, abl) == 0
    frags = [(ops.mfma_frag_layout(w.reshape(w.shape[0], -1)), b) for w, b in ((w1, b1), (w2, b2), (w3, b3))]
    us = timeit(fused)
    if not (abl & 7):
        f_out = fused().clone()
        assert torch.equal(f_out, unfused()), abl
    print(f"fused pf={pf} abl={abl}: {us:8.2f} us", flush=True)
assert lib.sat_bottleneck_set_experiment(2, 0) == 0
frags = [(ops.mfma_frag_layout(w.reshape(w.shape[0], -1)), b) for w, b in ((w1, b1), (w2, b2), (w3, b3))]
ref = unfused().clone()
out = fused()
torch.cuda.synchronize()
print("bit-identical:", torch.equal(ref, out), flush=True)

# whole trunk as one graph, fused blocks on / off
torch.manual_seed(0)
enc = sat_amd.Encoder("resnet152", dtype=torch.bfloat16).to(dev).eval()
imgs = torch.randn(B, 3, 224, 224, device=dev)
res = {}
for fuse in (False, True, False, True):
    enc.fuse_blocks = fuse
    with torch.no_grad():
        enc(imgs)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        with torch.no_grad():
            o = enc(imgs)
    for _ in range(3):
        gr.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        gr.replay()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 20 * 1e3
    res.setdefault(fuse, []).append((ms, o.clone()))
    print(f"trunk graph fuse={fuse}: {ms:.3f} ms per {B} images", flush=True)
    del gr
print("trunk outputs equal:", torch.equal(res[True][0][1], res[False][0][1]))
