"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py (runs on the GPU box, stdlib only).

usage: python tools/prof_summary.py PROF_DIR BENCH_LOG [OUT_JSON]

* the kernel-stats rows of the classes bench.py's roofline names (calls, average us);
* the bench line's own avg_launch_us beside rocprof's average for the dominant class's kernel;
* how much of the traced busy time had kernels of two or more queues running at once (the kernel trace's
  serialisation of the overlapped encoder / decoder streams);
then deletes the (large) kernel_trace.csv so only the stats travel back.
"""
import csv
import glob
import json
import os
import sys

KEYS = ("conv3x3_frag", "conv3x3_band", "conv1x1_frag", "conv1x1_stream", "conv_pipe", "conv_ws", "fast_gemm",
        "skinny", "attn_", "lstm_", "loss_", "adam", "zero_rows", "colsum")


def decoder_nonloop(rows, steps=26):
    """The last train step's decoder-side launches that are not per time step (mean_rows .. the last Adam):
    per kernel name + grid, calls and total us (the head / loss / weight-gradient GEMMs and the small ones)."""
    import collections
    rows = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    ad = [i for i, n in enumerate(names) if "adam" in n]
    mr = [i for i, n in enumerate(names) if "mean_rows" in n]
    # the last bf16 decoder forward (mean_rows<bf16>) whose step ends in an Adam before the next forward
    m = last_ad = None
    for i in reversed(mr):
        if "DF16b" not in names[i] and "bf16" not in names[i]:
            continue
        nxt = [j for j in ad if j > i]
        later = [j for j in mr if j > i]
        if nxt and (not later or nxt[0] < later[0]):
            m = i
            last_ad = max(j for j in ad if j > i and (not later or j < later[0]))
            break
    if m is None:
        return None
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rows[m:last_ad + 1]:
        n = r["Kernel_Name"]
        k = n[:100] + f" g={r.get('Grid_Size_X', r.get('Grid_Size', '?'))},{r.get('Grid_Size_Y', '')}"
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    out = [{"calls": c, "us": round(d, 1), "kernel": k} for k, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])
           if not (c >= steps and c % steps == 0)]
    return {"launches": sum(o["calls"] for o in out), "us": round(sum(o["us"] for o in out), 1), "top": out[:40]}


def main():
    d, log = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else None
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    trace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    res = {"kernels": []}
    if stats:
        for row in csv.DictReader(open(stats[0])):
            if any(k in row["Name"] for k in KEYS):
                res["kernels"].append({"name": row["Name"][:110], "calls": int(row["Calls"]),
                                       "avg_us": round(float(row["AverageNs"]) / 1e3, 3),
                                       "pct": float(row["Percentage"])})
    line = None
    for l in open(log):
        if l.startswith("{"):
            line = json.loads(l)
    if line and line.get("roofline"):
        r = line["roofline"]
        res["bench"] = {k: r.get(k) for k in ("cls", "avg_launch_us", "avg_launch_us_overlapped", "frac",
                                              "algorithmic_flops_per_launch")}
        kn = "conv3x3_frag" if "conv3x3_frag" in r.get("kernel", "") else None
        if kn:
            rows = [k for k in res["kernels"] if kn in k["name"]]
            if rows:
                avg = rows[0]["avg_us"]
                res["rocprof_dominant"] = {"kernel": rows[0]["name"], "avg_us": avg, "calls": rows[0]["calls"],
                                           "frac": round(r["algorithmic_flops_per_launch"] / (avg * 1e-6) / 2.5e15, 4),
                                           "bench_over_rocprof": round(r["avg_launch_us"] / avg, 4)}
    if trace:
        ev = []
        rows = []
        with open(trace[0]) as f:
            rd = csv.DictReader(f)
            for row in rd:
                q = row.get("Queue_Id") or row.get("Stream_Id") or "0"
                ev.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), q))
                rows.append(row)
        res["decoder_nonloop"] = decoder_nonloop(rows)
        pts = []
        for s, e, q in ev:
            pts.append((s, 1, q))
            pts.append((e, -1, q))
        pts.sort()
        active = {}
        busy = multi = 0
        last = None
        for t, dlt, q in pts:
            if last is not None:
                nq = sum(1 for v in active.values() if v > 0)
                if nq >= 1:
                    busy += t - last
                if nq >= 2:
                    multi += t - last
            active[q] = active.get(q, 0) + dlt
            last = t
        res["trace"] = {"kernels": len(ev), "queues": len({q for _, _, q in ev}),
                        "busy_ms": round(busy / 1e6, 2), "two_or_more_queues_ms": round(multi / 1e6, 2),
                        "overlap_frac": round(multi / busy, 4) if busy else None}
        os.remove(trace[0])
    s = json.dumps(res, indent=1)
    print(s)
    if out:
        open(out, "w").write(s)


if __name__ == "__main__":
    main()
