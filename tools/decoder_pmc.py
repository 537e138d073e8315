"""HBM traffic of the decoder's per-time-step kernels from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE),
against their algorithmic bytes (sat_amd.diagnostics.step_group_bytes).

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d F -o run --output-format csv -- python tools/decoder_pmc.py
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -d W -o run --output-format csv -- python tools/decoder_pmc.py
    python tools/decoder_pmc.py --analyze F W [out.json]

The run: the bench's decoder instance (B = 128, ResNet152 features L = 49 x D = 2048, E = 512, V = 10000, T = 27,
--attention --tf --ado, bf16, split target 96) train step, eager, three times.  Counters per MI355X_MICROARCH.md
§HBM: FETCH_SIZE x2 on gfx950 (16-B streaming reads), WRITE_SIZE as is; rocprofv3 reports both in KiB.
Per-step windows of the last forward / BPTT (middle steps): a forward window runs from the dispatch after one
attn_fwd to the next attn_fwd inclusive, a backward window likewise between two attention backwards, so each
holds one step's set of kernels whatever the launch count per step.
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

B, LF, D, E, V, T = 128, 49, 2048, 512, 10000, 27


def run():
    import torch
    import sat_amd
    from sat_amd.data import synthetic_captions
    torch.manual_seed(0)
    dev = "cuda"
    dec = sat_amd.Decoder(V, D, tf=True, ado=True, attention=True).to(dev).train()
    dec.split_target = int(os.environ.get("SAT_SPLIT_TARGET", "96"))   # bench.py's B = 128 instance
    dec.record_tokens = False
    opt = sat_amd.Adam(dec.parameters(), lr=1e-4)
    g = torch.Generator().manual_seed(1)
    feats = torch.randn(B, LF, D, generator=g).relu().bfloat16().to(dev)
    caps = synthetic_captions(B, T, V, generator=g, device=dev)
    for _ in range(3):
        opt.zero_grad()
        preds, alphas = dec(feats, caps)
        loss, _ = sat_amd.caption_loss(preds, alphas, caps)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    print("decoder_pmc: 3 train steps done, loss", float(loss))


def read_counter(d, name):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = {}
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") != name:
                    continue
                did = int(r["Dispatch_Id"])
                k, v = per.get(did, (r["Kernel_Name"], 0.0))
                per[did] = (k, v + float(r["Counter_Value"]))
    return [(k, v) for _, (k, v) in sorted(per.items())]


def short(name):
    """Kernel name without namespace, template arguments and parameters (demangled or Itanium-mangled)."""
    import re
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)", n)
    if m:
        k = int(m.group(1))
        return n[m.end():m.end() + k]
    return n.split("<")[0].split("(")[0]


def label(window, attn_key):
    """Group labels for one step window (kernel names; a GEMM right before the attention kernel is the h GEMM
    in the forward, the d(gated context) GEMM in the backward)."""
    out = []
    for i, (k, _) in enumerate(window):
        n = short(k)
        if "attn_fwd" in n:
            out.append("attn_fwd")
        elif "attn_bwd" in n:
            out.append("attn_bwd")
        elif "lstm_fwd" in n and "gemm" not in n:
            out.append("lstm_fwd")
        elif "lstm_bwd" in n and "gemm" not in n:
            out.append("lstm_bwd")
        elif "lstm_gemm_fwd" in n:
            out.append("ctx_gemm+lstm_fwd")
        elif "lstm_gemm_bwd" in n:
            out.append("dh_gemm+lstm_bwd")
        else:
            nxt = short(window[i + 1][0]) if i + 1 < len(window) else ""
            if attn_key == "attn_fwd":
                out.append("h_gemm" if "attn_fwd" in nxt else "ctx_gemm")
            else:
                out.append("dgated_gemm" if "attn_bwd" in nxt else "dh_gemm")
    return out


def windows(rows, key):
    idx = [i for i, (k, _) in enumerate(rows) if key in k]
    if len(idx) < 4:
        raise SystemExit(f"fewer than 4 {key} dispatches")
    # the last train step's loop: its T-1 attention launches are the last T-1 of them
    idx = idx[-(T - 1):]
    return [rows[a + 1:b + 1] for a, b in zip(idx, idx[1:])]


def analyze(fdir, wdir, out_path=None):
    from sat_amd.diagnostics import step_group_bytes
    alg = step_group_bytes(B, LF, D, E, T, 2, True, True)
    alg["ctx_gemm+lstm_fwd"] = alg["ctx_gemm"] + alg["lstm_fwd"]
    alg["dh_gemm+lstm_bwd"] = alg["dh_gemm"] + alg["lstm_bwd"]
    fetch, write = read_counter(fdir, "FETCH_SIZE"), read_counter(wdir, "WRITE_SIZE")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, --kernel-trace), "
                     "tools/decoder_pmc.py (eager decoder train step, bench instance); FETCH_SIZE x2 (gfx950), "
                     "KiB -> bytes; per launch = mean over the middle steps of the last train step",
           "shape": dict(B=B, L=LF, D=D, E=E, V=V, T=T, dtype="bf16", split_target=96), "groups": {}}
    for key in ("attn_fwd", "attn_bwd_split_kernel"):
        fw, ww = windows(fetch, key), windows(write, key)
        for wf, wwin in zip(fw[1:-1], ww[1:-1]):   # middle steps only
            labs = label(wf, "attn_fwd" if key == "attn_fwd" else "attn_bwd")
            for lab, (k, fv), (_, wv) in zip(labs, wf, wwin):
                g = res["groups"].setdefault(lab, {"kernel": short(k), "n": 0, "fetch": 0.0, "write": 0.0})
                g["n"] += 1
                g["fetch"] += fv * 2.0 * 1024
                g["write"] += wv * 1024
    tot_hbm = tot_alg = 0.0
    for lab, g in res["groups"].items():
        g["fetch_bytes_per_launch"] = round(g.pop("fetch") / g["n"])
        g["write_bytes_per_launch"] = round(g.pop("write") / g["n"])
        g["hbm_bytes_per_launch"] = g["fetch_bytes_per_launch"] + g["write_bytes_per_launch"]
        g["alg_bytes"] = alg.get(lab)
        if g["alg_bytes"]:
            g["ratio_to_algorithmic"] = round(g["hbm_bytes_per_launch"] / g["alg_bytes"], 3)
            tot_hbm += g["hbm_bytes_per_launch"]
            tot_alg += g["alg_bytes"]
    res["per_step_hbm_bytes"] = round(tot_hbm)
    res["per_step_alg_bytes"] = round(tot_alg)
    res["note"] = ("FETCH_SIZE counts Infinity-Cache (MALL) hits as fabric reads (MI355X_MICROARCH.md §HBM): the "
                   "annotation / Ws rows each step re-reads (~32 MB, resident in the 256 MB MALL) show up at full "
                   "size; a ratio well above 1 means re-fetches beyond that")
    print(json.dumps(res, indent=1))
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)


def counters(d, out_path=None):
    """Mean of every collected counter per kernel (short name) over the last train step's per-step dispatches
    (the last T-1 forward and T-1 backward windows); for the SQ / TCC groups of tools/session.sh pmcdec2."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    rows = {}
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                did = int(r["Dispatch_Id"])
                e = rows.setdefault(did, {"k": r["Kernel_Name"]})
                e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    seq = [rows[k] for k in sorted(rows)]
    last_fwd = max(i for i, e in enumerate(seq) if "attn_fwd" in e["k"])
    first = last_fwd - 40 * (T - 1)   # the last step's forward + backward: ~4-8 launches per time step each
    res = {}
    for e in seq[max(0, first):]:
        n = short(e["k"])
        if not any(x in n for x in ("attn_", "skinny", "lstm", "fast_gemm")):
            continue
        g = res.setdefault(n, {"n": 0})
        g["n"] += 1
        for c, v in e.items():
            if c != "k":
                g[c] = g.get(c, 0.0) + v
    for n, g in res.items():
        for c in list(g):
            if c != "n":
                g[c] = round(g[c] / g["n"], 1)
    print(json.dumps(res, indent=1))
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--counters":
        counters(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
    elif len(sys.argv) > 1 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else None)
    else:
        run()
