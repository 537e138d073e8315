"""Per-kernel time of the last decoder step (mean_rows .. last adam) in a rocprofv3 kernel trace.

    python tools/decoder_census.py <run_kernel_trace.csv> [top]
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
ad = [i for i, n in enumerate(names) if "adam" in n]
mr = [i for i, n in enumerate(names) if "mean_rows" in n]
last_ad = ad[-1]
m = max(i for i in mr if i < last_ad)
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows[m:last_ad + 1]:
    n = r["Kernel_Name"]
    k = (n[n.index("fast_gemm_kernel"):][:50] + f" g={r['Grid_Size_X']},{r['Grid_Size_Y']},{r['Grid_Size_Z']}"
         if "fast_gemm" in n else n[:60])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[k][0] += 1
    agg[k][1] += d
for k, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{n:4d} {d:8.1f}us avg {d / n:6.1f}  {k}")
span = (int(rows[last_ad]["End_Timestamp"]) - int(rows[m]["Start_Timestamp"])) / 1e3
print(f"decoder busy {sum(v[1] for v in agg.values()):.1f} us, span {span:.1f} us")
