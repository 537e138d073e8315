"""Per-kernel time per step of two rocprofv3 kernel_stats.csv files (A/B of two builds), largest differences first.
   python tools/prof_diff.py A.csv B.csv [steps]"""
import csv
import sys


def load(p):
    return {r["Name"]: (int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(p))}


a, b = load(sys.argv[1]), load(sys.argv[2])
steps = float(sys.argv[3]) if len(sys.argv) > 3 else 65.0
rows = []
for n in set(a) | set(b):
    ta, tb = a.get(n, (0, 0))[1] / steps / 1e3, b.get(n, (0, 0))[1] / steps / 1e3
    rows.append((ta - tb, ta, tb, n))
rows.sort()
for d, ta, tb, n in rows[:10] + rows[-10:]:
    print(f"{d:+8.1f} us  A {ta:8.1f}  B {tb:8.1f}  {n[:110]}")
print(f"total per step: A {sum(r[1] for r in rows):.1f} us  B {sum(r[2] for r in rows):.1f} us")
