"""A/B the kernel choice for single ResNet152 conv classes (GPU): each class's conv at B images re-issued back to
back between HIP events under several SatPolicy settings (conv_pipe / conv_stream / gemm_tile /
gemm_linear_order), outputs checked bit-identical to the default where the arithmetic order allows.

    python tools/conv_class_ab.py [B] [--only L4c2,...]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import sat_amd  # noqa: E402
from sat_amd import ops  # noqa: E402

DEV = torch.device("cuda")
B = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 128
# name, H (input), Cin, Cout, k, stride, pad, residual
CLASSES = [
    ("L4c2 3x3 512", 7, 512, 512, 3, 1, 1, False),
    ("L2c2 3x3 128", 28, 128, 128, 3, 1, 1, False),
    ("L3c2 3x3 256", 14, 256, 256, 3, 1, 1, False),
    ("L4c2s2 3x3 512 /2", 14, 512, 512, 3, 2, 1, False),
    ("L4c1 1x1 2048->512", 7, 2048, 512, 1, 1, 0, False),
    ("L4c3+res 1x1 512->2048", 7, 512, 2048, 1, 1, 0, True),
    ("L4dss2 1x1 1024->2048 /2", 14, 1024, 2048, 1, 2, 0, False),
    ("L3c2s2 3x3 256 /2", 28, 256, 256, 3, 2, 1, False),
    ("L3dss2 1x1 512->1024 /2", 28, 512, 1024, 1, 2, 0, False),
    ("V4 3x3 128 (VGG19 block 2)", 112, 128, 128, 3, 1, 1, False),
    ("V7 3x3 256 (VGG19 block 3)", 56, 256, 256, 3, 1, 1, False),
    ("V12 3x3 512 (VGG19 block 4)", 28, 512, 512, 3, 1, 1, False),
    ("V11 3x3 256->512 (VGG19 block 4)", 28, 256, 512, 3, 1, 1, False),
    ("V6 3x3 128->256 (VGG19 block 3)", 56, 128, 256, 3, 1, 1, False),
    ("V3 3x3 64->128 (VGG19 block 2)", 112, 64, 128, 3, 1, 1, False),
    ("V1 3x3 64 (VGG19 block 1)", 224, 64, 64, 3, 1, 1, False),
]
POLICIES = [("default", {}), ("pipe off", dict(conv_pipe=1)), ("pipe all", dict(conv_pipe=2)),
            ("tile1", dict(conv_pipe=1, gemm_tile=1)), ("tile2", dict(conv_pipe=1, gemm_tile=2)),
            ("tile4", dict(conv_pipe=1, gemm_tile=4)), ("tile5", dict(conv_pipe=1, gemm_tile=5)),
            ("linear order", dict(gemm_linear_order=1)), ("frag", dict(frag=True)),
            ("frag slices1", dict(frag=True, conv_slices=1)), ("frag slices2", dict(frag=True, conv_slices=2))]


def main():
    g = torch.Generator(device=DEV).manual_seed(0)
    only = sys.argv[sys.argv.index("--only") + 1].replace("/", ",").split(",") if "--only" in sys.argv else None
    for name, H, Cin, Cout, k, s, p, res in CLASSES:
        if only and name.split()[0] not in only:
            continue
        OH = (H + 2 * p - k) // s + 1
        x = torch.randn(B, H, H, Cin, device=DEV, generator=g).relu().bfloat16()
        w = (torch.randn(Cout, k, k, Cin, device=DEV, generator=g) * (2.0 / (k * k * Cin)) ** 0.5).bfloat16()
        b = 0.1 * torch.randn(Cout, device=DEV, generator=g)
        r = torch.randn(B, OH, OH, Cout, device=DEV, generator=g).bfloat16() if res else None
        flops = 2.0 * B * OH * OH * Cout * k * k * Cin
        ref = None
        line = f"{name:26s} M {B * OH * OH:6d} N {Cout:5d} K {k * k * Cin:5d}:"
        for label, pol in POLICIES:
            pol = dict(pol)
            frag = pol.pop("frag", False)
            policy = sat_amd.Policy(**pol)
            if frag and not (k == 3 and s == 1 and ops.conv3x3_frag_supported(H, H, Cin, torch.bfloat16)):
                continue
            try:
                wfr = (ops.mfma_frag_layout(w.reshape(Cout, -1)), b) if frag else None

                def go():
                    if frag:   # the staged-input 3x3 kernel (sat_conv3x3_frag)
                        return ops.conv3x3_frag(x, wfr, policy=policy)
                    return ops.conv2d_nhwc(x, w, b, s, p, True, residual=r, out_hw=(OH, OH), policy=policy)
                y = go()
                for _ in range(2):
                    go()
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(10):
                    go()
                en.record()
                en.synchronize()
                us = st.elapsed_time(en) / 10 * 1e3
                if ref is None:
                    ref = y
                same = "=" if torch.equal(y, ref) else f"~{(y.float() - ref.float()).abs().max().item():.1e}"
                line += f"  {label} {us:.1f}{same} ({flops / us / 1e6:.0f} TF/s)"
            except RuntimeError as exc:
                line += f"  {label} err({str(exc)[:30]})"
        print(line, flush=True)


if __name__ == "__main__":
    main()
