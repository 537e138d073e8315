"""Per-conv-shape efficiency of the ResNet152 trunk from a rocprofv3 kernel trace (last step)."""
import csv, collections, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
ad = [i for i, r in enumerate(rows) if 'adam_kernel' in r['Kernel_Name']]
seg = rows[ad[-5] + 1:ad[-1] + 1]
fast = [r for r in seg if 'fast_gemm' in r['Kernel_Name']]
def shapes(B=128):
    out = [("stem", B * 112 * 112, 64, 147, 0)]
    h, inpl = 56, 64
    for li, (n, pl) in enumerate(zip([3, 8, 36, 3], [64, 128, 256, 512])):
        for bi in range(n):
            s = (1 if li == 0 else 2) if bi == 0 else 1
            oh = h // s
            out.append((f"L{li+1}_c1", B * h * h, pl, inpl, 0))
            out.append((f"L{li+1}_c2", B * oh * oh, pl, 9 * pl, 0))
            if bi == 0:
                out.append((f"L{li+1}_ds", B * oh * oh, pl * 4, inpl, 0))
            out.append((f"L{li+1}_c3", B * oh * oh, pl * 4, pl, 1))
            inpl, h = pl * 4, oh
    return out
agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
for r, (name, M, N, K, res) in zip(fast, shapes()):
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    a = agg[f"{name} M={M} N={N} K={K}"]
    a[0] += 1; a[1] += d; a[2] += 2 * M * N * K
    a[3] += 2 * (M * N * (2 if res else 1) + M * K + N * K)
tot = 0
for k, (n, d, f, b) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    tot += d
    print(f"{k:36s} n={n:3d} {d:8.1f}us {f/d/1e6:7.1f} TF/s  {b/d/1e3:6.2f} TB/s(min bytes)")
print("conv total us", tot)
