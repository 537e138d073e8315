"""Per-step kernel census from a rocprofv3 kernel trace (one step = between consecutive Adam launches)."""
import collections, csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
ad = [i for i, r in enumerate(rows) if 'adam_kernel' in r['Kernel_Name']]
# last step: from the first adam launch of the previous step group to the last adam
groups = []
for i in ad:
    if groups and i - groups[-1][-1] <= 4:
        groups[-1].append(i)
    else:
        groups.append([i])
s, e = groups[-2][-1], groups[-1][-1]
seg = rows[s + 1:e + 1]
c = collections.Counter(); tot = collections.Counter()
for r in seg:
    k = r['Kernel_Name'].split('(')[0][:100]
    c[k] += 1; tot[k] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{c[k]:5d} {v/1e3:10.1f}us  {k}")
print("kernels", len(seg), "span ms", (int(seg[-1]['End_Timestamp']) - int(seg[0]['Start_Timestamp'])) / 1e6,
      "busy ms", sum(tot.values()) / 1e6)
