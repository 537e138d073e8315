"""HBM traffic per encoder conv class from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py <pmc_fetch dir> <pmc_write dir> [resnet152|vgg19] [B] [out.json]

Counters per MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports half the bytes of a wide
(16 B/lane) streaming read -> doubled here; WRITE_SIZE is exact for 16-B stores.  rocprofv3's
derived FETCH_SIZE / WRITE_SIZE are in KiB.  The input-layout conversion (a plain stream of known
size: B*3*224*224*4 B read; B*112*112*16*2 B written by the ResNet152 space-to-depth kernel,
B*224*224*8*2 by the VGG19 NHWC one) is reported beside them as the unit check.

Dispatch mapping as tools/conv_shapes.py: last complete encoder forward in each pass, its
fast_gemm_kernel dispatches in order onto bench.conv_launches().
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import conv_launches  # noqa: E402


CONV_KERNELS = ("fast_gemm_kernel", "conv_pipe_kernel", "conv1x1_stream_kernel",
                "bottleneck_kernel", "conv_ws_kernel", "conv3x3_frag_kernel", "conv3x3_half512_kernel", "conv3x3_band",
                "conv1x1_frag_kernel", "conv1x1_frag2_kernel", "conv3x3_slice2_kernel", "conv3x3_img_kernel",
                "block_band_kernel")


def is_conv_kernel(name):
    """A dispatch of one of the conv kernels bench.conv_launches() enumerates (one per launch)."""
    return any(k in name for k in CONV_KERNELS)


def read_counter(d, name):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = {}
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") != name:
                    continue
                did = int(r["Dispatch_Id"])
                k, v = per.get(did, (r["Kernel_Name"], 0.0))
                per[did] = (k, v + float(r["Counter_Value"]))
    return [(did, k, v) for did, (k, v) in sorted(per.items())]


def last_forward(rows, n_conv):
    groups, cur = [], None
    for did, k, v in rows:
        if "nchw_to_nhwc" in k or "s2d16" in k:   # the input layout kernel opens a forward
            cur = []
            groups.append(cur)
        elif "mean_rows" in k:
            cur = None
        if cur is not None:
            cur.append((k, v))
    groups = [g for g in groups if sum(is_conv_kernel(k) for k, _ in g) == n_conv]
    if not groups:
        raise SystemExit("no complete encoder forward")
    return groups[-1]


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    network = sys.argv[3] if len(sys.argv) > 3 else "resnet152"
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 128
    launches = conv_launches(network, B, fused=False)   # bench.py's default schedule: no block fused
    n = len(launches)
    out = {"source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes, --kernel-trace), "
                     "bench.py --no-graph; FETCH_SIZE x2 (gfx950), KiB -> bytes",
           "network": network, "batch": B, "classes": {}}
    fetch = last_forward(read_counter(fdir, "FETCH_SIZE"), n)
    write = last_forward(read_counter(wdir, "WRITE_SIZE"), n)
    unit = {}
    for tag, g, scale in (("fetch", fetch, 2.0), ("write", write, 1.0)):
        layout = [v for k, v in g if "nchw_to_nhwc" in k or "s2d16" in k]
        unit[tag] = layout[0] * scale * 1024 if layout else None
        conv = [v * scale * 1024 for k, v in g if is_conv_kernel(k)]
        for l, b in zip(launches, conv):
            c = out["classes"].setdefault(l["cls"], {"n": 0, "fetch": 0.0, "write": 0.0, "alg_bytes": l["bytes"]})
            if tag == "fetch":
                c["n"] += 1
            c[tag] += b
    tot = 0.0
    for name, c in out["classes"].items():
        c["hbm_bytes_per_launch"] = (c["fetch"] + c["write"]) / c["n"]
        c["ratio_to_algorithmic"] = round(c["hbm_bytes_per_launch"] / c["alg_bytes"], 3)
        tot += c["fetch"] + c["write"]
    out["hbm_bytes_encoder_convs"] = tot
    s2d = network == "resnet152"   # ResNet152: RGB -> 2x2 space-to-depth NHWC16 (stem as 4x4/s1 conv)
    out["unit_check_input_layout"] = {"kernel": "nchw3_to_s2d16" if s2d else "nchw_to_nhwc",
                                      "fetch_bytes": unit["fetch"], "expected_read": B * 3 * 224 * 224 * 4,
                                      "write_bytes": unit["write"],
                                      "expected_write": B * 112 * 112 * 16 * 2 if s2d else B * 224 * 224 * 8 * 2}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 5:
        with open(sys.argv[5], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
