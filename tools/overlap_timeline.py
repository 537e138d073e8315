"""Overlapped-step timeline from a rocprofv3 kernel trace of bench.py (graph mode): per stream, the
kernels' busy time, span and idle gaps inside the last complete steps, and per kernel class the
average duration -- to see what the decoder chain loses beside the encoder trunk.
    rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python bench.py --steps 20 ...
    python tools/overlap_timeline.py DIR/run_kernel_trace.csv [steps]"""
import collections
import csv
import sys


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")
    n = n.replace("_GLOBAL__N_1", "")
    return n[:70]


def main():
    path = sys.argv[1]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    rows = list(csv.DictReader(open(path)))
    cols = rows[0].keys()
    skey = "Stream_Id" if "Stream_Id" in cols else ("Queue_Id" if "Queue_Id" in cols else None)
    print("columns:", ",".join(cols))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    # one Adam launch per step (fused flat buffer): the last nsteps steps
    groups = []
    for i in adam:
        if groups and i - groups[-1][-1] <= 4:
            groups[-1].append(i)
        else:
            groups.append([i])
    if len(groups) < nsteps + 1:
        raise SystemExit(f"{len(groups)} Adam groups, need {nsteps + 1}")
    s, e = groups[-nsteps - 1][-1], groups[-1][-1]
    t0, t1 = int(rows[s]["End_Timestamp"]), int(rows[e]["End_Timestamp"])
    seg = [r for r in rows[s + 1:e + 1]]
    print(f"{nsteps} steps: {(t1 - t0) / nsteps / 1e3:.1f} us/step, {len(seg) / nsteps:.0f} kernels/step")
    by_stream = collections.defaultdict(list)
    for r in seg:
        by_stream[r[skey] if skey else "all"].append(r)
    for sid, rs in by_stream.items():
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs)
        # union of kernel intervals (overlapping kernels on one stream are graph branches)
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rs)
        cover, cs, ce = 0, iv[0][0], iv[0][1]
        for a, b in iv[1:]:
            if a > ce:
                cover += ce - cs
                cs, ce = a, b
            else:
                ce = max(ce, b)
        cover += ce - cs
        names = collections.Counter(short(r["Kernel_Name"]) for r in rs)
        print(f"\nstream {sid}: {len(rs) / nsteps:.0f} kernels/step, busy {busy / nsteps / 1e3:.1f} us/step, "
              f"covered {cover / nsteps / 1e3:.1f} us/step, top: {names.most_common(3)}")
        dur = collections.defaultdict(list)
        for r in rs:
            dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1]))[:14]:
            print(f"   {k:70s} {len(v) / nsteps:6.1f}/step {sum(v) / nsteps / 1e3:8.1f} us/step avg {sum(v) / len(v) / 1e3:7.2f}")
        # gaps between consecutive kernels of this stream (dispatch waits + launch boundaries)
        gaps = [max(0, int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) for a, b in zip(rs, rs[1:])]
        gaps.sort()
        if gaps:
            print(f"   gaps: sum {sum(gaps) / nsteps / 1e3:.1f} us/step, median {gaps[len(gaps) // 2] / 1e3:.2f} us, "
                  f"p90 {gaps[int(len(gaps) * 0.9)] / 1e3:.2f} us, max {gaps[-1] / 1e3:.1f} us")


if __name__ == "__main__":
    main()
