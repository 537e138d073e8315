"""HBM traffic of the encoder's conv launches from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py gpurun_out/<tag>/pmc_fetch gpurun_out/<tag>/pmc_write [out.json]

Counters follow MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of a wide (16 B/lane)
streaming read on gfx950 -> doubled here; WRITE_SIZE is exact for 16-B stores.  Both are in KiB
per dispatch (rocprofv3 derived-counter unit); the NCHW->NHWC input conversion (a pure stream of
known size) is printed beside them as a unit/calibration check.

Encoder dispatches = from each ``nchw_to_nhwc_kernel`` up to the decoder's first
``mean_rows_kernel``; the conv launches among them are the ``fast_gemm_kernel`` ones.
"""
import csv
import glob
import json
import os
import sys


def read_counter(d, name):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") == name:
                    rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    # one value per dispatch (sum over per-XCD / per-instance rows if any)
    out = {}
    for did, k, v in rows:
        if did in out:
            out[did] = (k, out[did][1] + v)
        else:
            out[did] = (k, v)
    return [(did, k, v) for did, (k, v) in sorted(out.items())]


def encoder_groups(rows):
    groups, cur = [], None
    for did, k, v in rows:
        if "nchw_to_nhwc" in k:
            cur = []
            groups.append(cur)
        elif "mean_rows" in k:
            cur = None
        if cur is not None:
            cur.append((did, k, v))
    return groups


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    out_path = sys.argv[3] if len(sys.argv) > 3 else None
    fetch = read_counter(fdir, "FETCH_SIZE")
    write = read_counter(wdir, "WRITE_SIZE")
    res = {}
    for name, rows, scale in (("fetch", fetch, 2.0), ("write", write, 1.0)):
        gs = [g for g in encoder_groups(rows) if g]
        g = gs[-1]   # last (steady-state) encoder forward
        conv = [v for _, k, v in g if "fast_gemm_kernel" in k]
        layout = [v for _, k, v in g if "nchw_to_nhwc" in k]
        res[name] = dict(encoder_forwards_seen=len(gs), conv_launches=len(conv),
                         conv_kib_total=sum(conv) * scale, conv_kib_per_launch=sum(conv) * scale / max(1, len(conv)),
                         nchw_to_nhwc_kib=(layout[0] * scale if layout else None), scale_applied=scale)
    n = res["fetch"]["conv_launches"]
    per_launch = (res["fetch"]["conv_kib_total"] + res["write"]["conv_kib_total"]) * 1024 / max(1, n)
    summary = dict(source="rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), --kernel-trace, "
                          "bench.py --no-graph; FETCH_SIZE x2 (gfx950 correction)",
                   conv_launches=n, hbm_bytes_per_conv_launch=per_launch,
                   hbm_bytes_encoder_convs=per_launch * n, detail=res)
    print(json.dumps(summary, indent=1))
    if out_path:
        with open(out_path, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
