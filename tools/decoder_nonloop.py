"""Per-kernel time of the last decoder step's kernels that are NOT per-time-step (the batched head,
loss, weight gradients, Adam) in a rocprofv3 kernel trace.

    python tools/decoder_nonloop.py <run_kernel_trace.csv> [T-1]
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 26
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
ad = [i for i, n in enumerate(names) if "adam" in n]
mr = [i for i, n in enumerate(names) if "mean_rows" in n]
last_ad = ad[-1]
m = max(i for i in mr if i < last_ad)
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows[m:last_ad + 1]:
    n = r["Kernel_Name"]
    k = (n[n.index("fast_gemm_kernel"):][:60] + f" g={r['Grid_Size_X']},{r['Grid_Size_Y']},{r['Grid_Size_Z']}"
         if "fast_gemm" in n else n[:70])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[k][0] += 1
    agg[k][1] += d
tot = 0.0
for k, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    if n >= steps and n % steps == 0:
        continue
    tot += d
    print(f"{n:4d} {d:8.1f}us  {k}")
print(f"non-loop total {tot:.1f} us")
