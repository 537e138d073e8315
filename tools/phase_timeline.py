"""Diagnostics: the decoder stream's phases per train step from a rocprofv3 kernel trace of bench.py (overlapped or
not): forward prologue, time loop, head + loss, backward phase 1, BPTT loop, phase-2 tail, Adam, and the gaps
between steps -- median microseconds over the traced steps.   python tools/phase_timeline.py run_kernel_trace.csv"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
adam_q = {r["Queue_Id"] for r in rows if "adam_kernel" in r["Kernel_Name"]}
dq = [r for r in rows if r["Queue_Id"] in adam_q]
other = [r for r in rows if r["Queue_Id"] not in adam_q]


def t0(r):
    return int(r["Start_Timestamp"]) / 1e3


def t1(r):
    return int(r["End_Timestamp"]) / 1e3


# steps: delimited by the decoder forward's first kernel (the caption embedding gather)
starts = [i for i, r in enumerate(dq) if "embed_gather_captions" in r["Kernel_Name"]]
phases = {}
for a, b in zip(starts, starts[1:]):
    step = dq[a:b]
    names = [r["Kernel_Name"] for r in step]

    def first(pred, lo=0):
        for i in range(lo, len(step)):
            if pred(names[i]):
                return i
        return None

    def last(pred):
        for i in range(len(step) - 1, -1, -1):
            if pred(names[i]):
                return i
        return None
    i_lf0 = first(lambda n: "lstm_fwd" in n)
    i_lf1 = last(lambda n: "lstm_fwd" in n)
    i_lb = first(lambda n: "loss_bwd" in n)
    i_b0 = first(lambda n: "lstm_bwd" in n)
    i_b1 = last(lambda n: "attn_bwd" in n)
    i_ad0 = first(lambda n: "adam_kernel" in n)
    if None in (i_lf0, i_lf1, i_lb, i_b0, i_b1, i_ad0):
        continue
    cut = {"fwd prologue": (0, i_lf0 - 3), "time loop fwd": (i_lf0 - 3, i_lf1), "head + loss": (i_lf1 + 1, i_lb),
           "bwd phase 1": (i_lb + 1, i_b0 - 1), "BPTT loop": (i_b0 - 1, i_b1 + 1), "phase-2 tail": (i_b1 + 2, i_ad0 - 1),
           "Adam": (i_ad0, len(step) - 1)}
    for k, (x, y) in cut.items():
        x = max(0, min(x, len(step) - 1)); y = max(x, min(y, len(step) - 1))
        phases.setdefault(k, []).append(t1(step[y]) - t0(step[x]))
    phases.setdefault("step (start to next start)", []).append(t0(dq[b]) - t0(step[0]))
    busy = sum(t1(r) - t0(r) for r in step)
    phases.setdefault("decoder kernels busy", []).append(busy)
for k, v in phases.items():
    print(f"{k:28s} {statistics.median(v):9.1f} us  (n={len(v)})")
