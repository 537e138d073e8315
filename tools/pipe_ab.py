"""A/B the 256x128 pipelined conv kernel (convpipe.hip) and the 1x1 streaming kernel (convstream.hip),
both forced on (mode 2), against the 128-row LDS-DMA kernel (convgemm.hip, both mode 0) on the ResNet152 / VGG19 conv shapes at B=128.
Interleaved rounds in one process (cdna_hip_programming.md 5.4 rule 24); median of rounds.
Also checks that both kernels give bit-identical outputs (same fp32 sums, same rounding)."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import sat_amd  # noqa: E402
from sat_amd import ops  # noqa: E402

B = int(os.environ.get("B", "128"))
REPS = int(os.environ.get("REPS", "10"))
# (name, H, Cin, Cout, k, stride, pad, residual)
SHAPES = [("L3_c2", 14, 256, 256, 3, 1, 1, 0), ("L3_c1", 14, 1024, 256, 1, 1, 0, 0),
          ("L3_c3", 14, 256, 1024, 1, 1, 0, 1), ("L2_c2", 28, 128, 128, 3, 1, 1, 0),
          ("L2_c1", 28, 512, 128, 1, 1, 0, 0), ("L2_c3", 28, 128, 512, 1, 1, 0, 1),
          ("L4_c2", 7, 512, 512, 3, 1, 1, 0), ("L4_c1", 7, 2048, 512, 1, 1, 0, 0),
          ("L4_c3", 7, 512, 2048, 1, 1, 0, 1), ("L1_c2", 56, 64, 64, 3, 1, 1, 0),
          ("L3_c2s2", 28, 256, 256, 3, 2, 1, 0), ("L4_c1a", 14, 1024, 512, 1, 1, 0, 0),
          ("vgg_c512", 28, 512, 512, 3, 1, 1, 0), ("vgg_c256", 56, 256, 256, 3, 1, 1, 0),
          ("vgg_c14", 14, 512, 512, 3, 1, 1, 0), ("vgg_c128", 112, 128, 128, 3, 1, 1, 0),
          ("L1_c3", 56, 64, 256, 1, 1, 0, 1), ("L1_ds", 56, 64, 256, 1, 1, 0, 0), ("L1_c1", 56, 256, 64, 1, 1, 0, 0),
          ("L2_dss2", 56, 256, 512, 1, 2, 0, 0), ("L3_dss2", 28, 512, 1024, 1, 2, 0, 0),
          ("L4_dss2", 14, 1024, 2048, 1, 2, 0, 0), ("L2_c1a", 56, 256, 128, 1, 1, 0, 0)]
ONLY = os.environ.get("SHAPES")
if ONLY:
    SHAPES = [t for t in SHAPES if t[0] in ONLY.split(",")]
lib = sat_amd._lib.lib()
torch.manual_seed(0)
for name, H, C, Co, k, s, p, r in (SHAPES if not (os.environ.get("EXP") or os.environ.get("SABL")) else []):
    x = torch.randn(B, H, H, C, device="cuda").bfloat16()
    w = (torch.randn(Co, k, k, C, device="cuda") / (k * k * C) ** 0.5).bfloat16()
    b = torch.randn(Co, device="cuda")
    OH = (H + 2 * p - k) // s + 1
    resid = torch.randn(B, OH, OH, Co, device="cuda").bfloat16() if r else None
    outs = {}
    for mode in (0, 2):
        lib.sat_conv_pipe_set_mode(mode)
        lib.sat_conv_stream_set_mode(mode)
        lib.sat_conv_halo_set_mode(mode)
        outs[mode] = ops.conv2d_nhwc(x, w, b, s, p, True, residual=resid)
    same = torch.equal(outs[0], outs[2])
    maxdiff = (outs[0].float() - outs[2].float()).abs().max().item()
    y = outs[0]
    flops = 2.0 * B * OH * OH * Co * k * k * C
    times = {0: [], 2: []}
    for rnd in range(5):
        for mode in (0, 2):
            lib.sat_conv_pipe_set_mode(mode)
            lib.sat_conv_stream_set_mode(mode)
            lib.sat_conv_halo_set_mode(mode)
            ops.conv2d_nhwc(x, w, b, s, p, True, residual=resid, out=y)
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(REPS):
                ops.conv2d_nhwc(x, w, b, s, p, True, residual=resid, out=y)
            en.record()
            en.synchronize()
            times[mode].append(st.elapsed_time(en) / REPS)
    lib.sat_conv_pipe_set_mode(1)
    lib.sat_conv_stream_set_mode(1)
    lib.sat_conv_halo_set_mode(1)
    t0, t2 = statistics.median(times[0]), statistics.median(times[2])
    print(f"{name:9s} M={B*OH*OH:7d} N={Co:5d} K={k*k*C:5d}  old {t0*1e3:7.1f}us {flops/t0/1e9:5.0f}TF  "
          f"pipe {t2*1e3:7.1f}us {flops/t2/1e9:5.0f}TF  x{t0/t2:4.2f}  bitequal={same} maxdiff={maxdiff:.3g}",
          flush=True)

# ---- plain NT GEMMs (decoder shapes): C bf16 = relu(A B^T + bias)
GEMMS = [(3328, 10000, 512), (6272, 512, 2048), (3328, 2048, 512), (6272, 768, 512), (4096, 30522, 768)]
for M, N, K in (GEMMS if not (os.environ.get("EXP") or os.environ.get("SABL")) and not ONLY else []):
    A = torch.randn(M, K, device="cuda").bfloat16()
    Wt = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    bias = torch.randn(N, device="cuda")
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    outs, times = {}, {0: [], 2: []}
    for rnd in range(5):
        for mode in (0, 2):
            lib.sat_conv_pipe_set_mode(mode)
            ops.gemm(A, Wt, C, bias=bias, act=sat_amd._lib.ACT_RELU)
            if rnd == 0:
                outs[mode] = C.clone()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(REPS):
                ops.gemm(A, Wt, C, bias=bias, act=sat_amd._lib.ACT_RELU)
            en.record()
            en.synchronize()
            times[mode].append(st.elapsed_time(en) / REPS)
    lib.sat_conv_pipe_set_mode(1)
    t0, t2 = statistics.median(times[0]), statistics.median(times[2])
    fl = 2.0 * M * N * K
    print(f"gemm {M}x{N}x{K}  old {t0*1e3:7.1f}us {fl/t0/1e9:5.0f}TF  pipe {t2*1e3:7.1f}us {fl/t2/1e9:5.0f}TF  "
          f"x{t0/t2:4.2f} bitequal={torch.equal(outs[0], outs[2])}", flush=True)

# ---- streaming-kernel ablation: SABL="0;1;2;4;3" (mode bits 2-4 of sat_conv_stream_set_mode)
SABL = os.environ.get("SABL")
if SABL:
    abls = [int(v) for v in SABL.split(";")]
    for name, H, C, Co, k, s, p, r in SHAPES:
        x = torch.randn(B, H, H, C, device="cuda").bfloat16()
        w = (torch.randn(Co, k, k, C, device="cuda") / (k * k * C) ** 0.5).bfloat16()
        b = torch.randn(Co, device="cuda")
        OH = (H + 2 * p - k) // s + 1
        resid = torch.randn(B, OH, OH, Co, device="cuda").bfloat16() if r else None
        y = torch.empty(B, OH, OH, Co, device="cuda", dtype=torch.bfloat16)
        times = {c: [] for c in abls}
        for rnd in range(5):
            for c in abls:
                lib.sat_conv_stream_set_mode(2 + 4 * c)
                ops.conv2d_nhwc(x, w, b, s, p, True, residual=resid, out=y)
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(REPS):
                    ops.conv2d_nhwc(x, w, b, s, p, True, residual=resid, out=y)
                en.record()
                en.synchronize()
                times[c].append(st.elapsed_time(en) / REPS)
        lib.sat_conv_stream_set_mode(1)
        print(f"{name:9s}" + "".join(f"  abl{c}: {statistics.median(times[c])*1e3:6.1f}us" for c in abls), flush=True)

# ---- experiment configs: EXP="8,0;4,0;8,1;8,2;8,4" (waves, ablation bits) on SHAPES, pipe forced
EXP = os.environ.get("EXP")
if EXP:
    cfgs = [tuple(int(v) for v in c.split(",")) for c in EXP.split(";")]
    lib.sat_conv_pipe_set_mode(2)
    for name, H, C, Co, k, s, p, r in SHAPES:
        if r:
            continue
        x = torch.randn(B, H, H, C, device="cuda").bfloat16()
        w = (torch.randn(Co, k, k, C, device="cuda") / (k * k * C) ** 0.5).bfloat16()
        b = torch.randn(Co, device="cuda")
        OH = (H + 2 * p - k) // s + 1
        y = torch.empty(B, OH, OH, Co, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * B * OH * OH * Co * k * k * C
        times = {c: [] for c in cfgs}
        ref = None
        for rnd in range(5):
            for c in cfgs:
                assert lib.sat_conv_pipe_set_experiment(*c) == 0
                ops.conv2d_nhwc(x, w, b, s, p, True, out=y)
                if c[1] == 0:
                    if ref is None:
                        ref = y.clone()
                    elif not torch.equal(ref, y):
                        print("MISMATCH", name, c, flush=True)
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(REPS):
                    ops.conv2d_nhwc(x, w, b, s, p, True, out=y)
                en.record()
                en.synchronize()
                times[c].append(st.elapsed_time(en) / REPS)
        lib.sat_conv_pipe_set_experiment(8, 0)
        line = f"{name:9s}"
        for c in cfgs:
            t = statistics.median(times[c])
            line += f"  w{c[0]}/a{c[1]} {t*1e3:6.1f}us {flops/t/1e9:5.0f}TF"
        print(line, flush=True)
    lib.sat_conv_pipe_set_mode(1)
