"""Per-conv-class timing of the encoder trunk from a rocprofv3 kernel trace.

    python tools/conv_shapes.py <run_kernel_trace.csv> [resnet152|vgg19] [B] [out.json]

Takes the last complete encoder forward in the trace (``nchw_to_nhwc`` or ``*_s2d16`` .. the decoder's first
``mean_rows``), maps its ``fast_gemm_kernel`` dispatches in order onto bench.conv_launches()
(the same class names and algorithmic bytes/FLOPs bench.py reports) and prints the average
launch duration and achieved rate per class -- the numbers bench.py's roofline must agree with.
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import conv_launches, BF16_DENSE_PEAK_TFLOPS, HBM_PEAK_GBS  # noqa: E402


CONV_KERNELS = ("fast_gemm_kernel", "conv_pipe_kernel", "conv1x1_stream_kernel", "bottleneck_kernel",
                "conv_ws_kernel", "conv3x3_frag_kernel", "conv3x3_half512_kernel", "conv3x3_band", "conv1x1_frag_kernel")


def is_conv_kernel(name):
    """A dispatch of one of the conv kernels bench.conv_launches() enumerates (one per launch)."""
    return any(k in name for k in CONV_KERNELS)


def encoder_dispatches(rows):
    groups, cur = [], None
    for r in rows:
        k = r["Kernel_Name"]
        if "nchw_to_nhwc" in k or "s2d16" in k:   # the input layout kernel opens a forward
            cur = []
            groups.append(cur)
        elif "mean_rows" in k:
            cur = None
        if cur is not None:
            cur.append(r)
    return groups


def main():
    path = sys.argv[1]
    network = sys.argv[2] if len(sys.argv) > 2 else "resnet152"
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    launches = conv_launches(network, B)
    groups = [g for g in encoder_dispatches(rows) if sum(is_conv_kernel(r["Kernel_Name"]) for r in g) == len(launches)]
    if not groups:
        raise SystemExit("no complete encoder forward in the trace")
    conv = [r for r in groups[-1] if is_conv_kernel(r["Kernel_Name"])]
    cls = {}
    for r, l in zip(conv, launches):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3   # us
        c = cls.setdefault(l["cls"], dict(n=0, us=0.0, flops=l["flops"], bytes=l["bytes"], bound=l["bound"]))
        c["n"] += 1
        c["us"] += d
    total = 0.0
    out = {}
    for name, c in sorted(cls.items(), key=lambda kv: -kv[1]["us"]):
        avg = c["us"] / c["n"]
        total += c["us"]
        tf = c["flops"] / (avg * 1e-6) / 1e12
        gbs = c["bytes"] / (avg * 1e-6) / 1e9
        frac = gbs / HBM_PEAK_GBS if c["bound"] == "hbm" else tf / BF16_DENSE_PEAK_TFLOPS
        out[name] = dict(n=c["n"], total_us=round(c["us"], 1), avg_launch_us=round(avg, 2), tflops=round(tf, 1),
                         gbs=round(gbs, 0), bound=c["bound"], frac=round(frac, 4))
        print(f"{name:28s} n={c['n']:3d} total {c['us']:8.1f}us avg {avg:7.2f}us {tf:7.1f} TF/s {gbs:7.0f} GB/s "
              f"[{c['bound']}] frac {frac:.3f}")
    print(f"conv total {total:.1f} us per forward ({len(groups)} complete forwards in trace)")
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            json.dump(dict(source=path, network=network, batch=B, conv_us_per_forward=round(total, 1), classes=out),
                      f, indent=1)


if __name__ == "__main__":
    main()
