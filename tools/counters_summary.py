"""Summarise tools/counters.sh output: per shape, the mean of each counter over the conv dispatches.

    python tools/counters_summary.py OUTDIR
"""
import collections
import csv
import glob
import os
import sys

out = sys.argv[1]
res = collections.defaultdict(dict)
for f in sorted(glob.glob(os.path.join(out, "*", "**", "*counter_collection.csv"), recursive=True)):
    shape = os.path.relpath(f, out).split(os.sep)[0].rsplit("_", 1)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if os.environ.get("KFILTER", "fast_gemm") not in r["Kernel_Name"]:
            continue
        per[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    for c, d in per.items():
        res[shape][c] = sum(d.values()) / len(d)
for shape, cs in res.items():
    print(shape)
    for c in sorted(cs):
        print(f"  {c:28s} {cs[c]:.4g}")
    w = cs.get("SQ_WAVE_CYCLES")
    if w:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in cs:
                print(f"  {c} / WAVE_CYCLES = {cs[c] / w:.3f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in cs and "GRBM_GUI_ACTIVE" in cs:
        print(f"  MFMA busy / (GUI_ACTIVE x 256 CUs x 4 SIMD) = "
              f"{cs['SQ_VALU_MFMA_BUSY_CYCLES'] / (cs['GRBM_GUI_ACTIVE'] / 8 * 256 * 4):.3f} (if BUSY counts per SIMD)")
