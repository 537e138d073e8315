"""Per-kernel-class time per step from a rocprofv3 kernel trace of bench.py: the last N steps, a step
starting at each encoder input-layout kernel (one per forward).  Class = (kernel, grid, LDS, VGPRs).
    python tools/trace_classes.py DIR/run_kernel_trace.csv [N] [top]"""
import collections
import csv
import re
import sys


def name(s):
    m = re.search(r"(\w+_kernel\w*)", s) or re.search(r"(\w+)\s*[<(]", s)
    return (m.group(1) if m else s)[:44]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "nchw3_to_s2d16" in r["Kernel_Name"] or "images_to_input" in r["Kernel_Name"]]
    seg = rows[marks[-n - 1]:marks[-1]]
    agg = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        k = (name(r["Kernel_Name"]), int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), int(r["Grid_Size_Y"]),
             int(r["LDS_Block_Size"]), int(r["VGPR_Count"]))
        agg[k][0] += 1
        agg[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot = sum(v[1] for v in agg.values())
    span = int(rows[marks[-1]]["Start_Timestamp"]) - int(seg[0]["Start_Timestamp"])
    print(f"{n} steps: kernel time {tot / n / 1e3:.1f} us/step, span {span / n / 1e3:.1f} us/step")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{v[1] / n / 1e3:8.1f} us/step {v[0] / n:5.1f}x avg {v[1] / v[0] / 1e3:7.2f}  {k}")


if __name__ == "__main__":
    main()
