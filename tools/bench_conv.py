"""A/B the bf16 LDS-DMA conv kernel configs (ring depth x tile x XCD remap) on the ResNet152 conv shapes (B=128).
Interleaved rounds in one process (cdna_hip_programming.md 5.4 rule 24); median of rounds."""
import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import sat_amd
from sat_amd import ops

B = int(os.environ.get("B", "128"))
dev = "cuda"
# (name, H, Cin, Cout, k, stride, pad, residual)
SHAPES = [("L1_c1", 56, 256, 64, 1, 1, 0, 0), ("L1_c2", 56, 64, 64, 3, 1, 1, 0), ("L1_c3", 56, 64, 256, 1, 1, 0, 1),
          ("L2_c2", 28, 128, 128, 3, 1, 1, 0), ("L2_c3", 28, 128, 512, 1, 1, 0, 1), ("L2_c1", 28, 512, 128, 1, 1, 0, 0),
          ("L3_c1", 14, 1024, 256, 1, 1, 0, 0), ("L3_c2", 14, 256, 256, 3, 1, 1, 0), ("L3_c3", 14, 256, 1024, 1, 1, 0, 1),
          ("L4_c2", 7, 512, 512, 3, 1, 1, 0), ("stem", 224, 8, 64, 7, 2, 3, 0)]
# (stages, tile, xcd_remap); tile ids: 1 128x128/8w, 2 128x64/8w, 3 128x128/4w, 4 128x256/8w, 5 256x128/8w
ONLY = os.environ.get("SHAPES")
if ONLY:
    SHAPES = [t for t in SHAPES if t[0] in ONLY.split(",")]
CONFIGS = [tuple(int(v) for v in c.split(',')) for c in os.environ.get('CONFIGS', '2,1,1;3,2,1;2,2,1').split(';')]
TNAME = {1: "128x128w8", 2: "128x64w8", 3: "128x128w4", 4: "128x256w8", 5: "256x128w8"}
lib = sat_amd._lib.lib()
res = {}
for name, H, C, Co, k, s, p, r in SHAPES:
    x = torch.randn(B, H, H, C, device=dev).bfloat16()
    w = (torch.randn(Co, k, k, C, device=dev) / (k * k * C) ** 0.5).bfloat16()
    b = torch.randn(Co, device=dev)
    OH = (H + 2 * p - k) // s + 1
    resid = torch.randn(B, OH, OH, Co, device=dev).bfloat16() if r else None
    y = torch.empty(B, OH, OH, Co, device=dev, dtype=torch.bfloat16)
    flops = 2.0 * B * OH * OH * Co * k * k * (3 if C == 8 else C)
    times = {c: [] for c in CONFIGS}
    for rnd in range(5):
        for cfg in CONFIGS:
            lib.sat_fast_gemm_set_config(*cfg[:3])
            if len(cfg) > 3:
                lib.sat_fast_gemm_set_res_lds(cfg[3])
            ops.conv2d_nhwc(x, w, b, s, p, True, residual=resid, out=y)
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(5):
                ops.conv2d_nhwc(x, w, b, s, p, True, residual=resid, out=y)
            en.record(); en.synchronize()
            times[cfg].append(st.elapsed_time(en) / 5)
    lib.sat_fast_gemm_set_config(0, 0, 1)
    if any(len(c) > 3 for c in CONFIGS):
        lib.sat_fast_gemm_set_res_lds(1)
    line = f"{name:6s} M={B*OH*OH:7d} N={Co:5d} K={k*k*C:5d} "
    for cfg in CONFIGS:
        ms = statistics.median(times[cfg])
        line += f" {TNAME.get(cfg[1], 'auto')}/s{cfg[0]}/x{cfg[2]}{'/e%d' % cfg[3] if len(cfg) > 3 else ''}:{ms*1e3:6.1f}us/{flops/ms/1e9:4.0f}TF"
    print(line, flush=True)
