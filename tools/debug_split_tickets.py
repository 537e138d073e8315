"""Ticket draws of the split-K GEMM inside the decoder's backward (GPU diagnosis; needs the diagnostics library
libsat_hip_sdbg.so: SAT_HIP_LIB_TUNING=show-attend-and-tell_amd/libsat_hip_sdbg.so).  Runs the deferred bf16
backward of tests/test_gpu_api.py's shape a number of times and prints, per launch, any tile whose S draws are not
0 .. S-1."""
import ctypes
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import sat_amd as sat  # noqa: E402
from oracle import sat_oracle as O  # noqa: E402

DEV = "cuda"
V, D, Lf, E, B, T = 60, 64, 16, 512, 3, 7
p = O.make_decoder_params(V, D, E, True, 5)
rng = np.random.default_rng(5)
feats = torch.from_numpy(rng.standard_normal((B, Lf, D)).astype(np.float32)).to(DEV).bfloat16()
caps = O.make_captions(B, T, V, 6).to(DEV)
dec = sat.Decoder(V, D, tf=True, ado=True, attention=True)
dec.load_state_dict(p, strict=True)
dec = dec.to(DEV).train()
dec.dropout_mask = torch.ones(B, T - 1, 512, dtype=torch.uint8, device=DEV)
lib = sat._lib.lib()
lib.sat_split_debug_read.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
buf = (ctypes.c_uint * (4 << 18))()
cnt = ctypes.c_uint(0)


def step():
    dec.zero_grad(set_to_none=True)
    dec.policy = sat.Policy(decoder_splits=[2, 2, 2, 2])
    preds, alphas = dec(feats, caps)
    sat.caption_loss(preds, alphas, caps)[0].backward()
    torch.cuda.synchronize()
    return {n: q.grad.detach().clone() for n, q in dec.named_parameters() if q.grad is not None}


lib.sat_split_debug_read(buf, 0, ctypes.byref(cnt))
cs = (ctypes.c_uint * (64 * 256))()
lib.sat_split_debug_checksums(cs)
runs = []
recs = []
sums = []
for r in range(16):
    runs.append(step())
    lib.sat_split_debug_read(buf, len(buf), ctypes.byref(cnt))
    n = min(cnt.value, len(buf) // 4)
    recs.append([tuple(buf[4 * i:4 * i + 4]) for i in range(n)])
    lib.sat_split_debug_checksums(cs)
    ls = sorted({rec[0] for rec in recs[-1]})
    sums.append([tuple(cs[(ln % 64) * 256 + t] for t in range(4)) for ln in ls])
ref = runs[-1]
for r, (g, rec) in enumerate(zip(runs, recs)):
    err = max(((g[n] - ref[n]).abs().max() / ref[n].abs().max()).item() for n in ("attention.U.weight", "init_h.weight"))
    by = defaultdict(list)
    for launch, tile, split, prev in rec:
        by[(launch, tile)].append((split, prev))
    launches = sorted({k[0] for k in by})
    # per launch (in order) the split that drew the last ticket, tile by tile
    last = []
    for ln in launches:
        tiles = sorted(t for (l2, t) in by if l2 == ln)
        last.append("".join(str(max(by[(ln, t)], key=lambda x: x[1])[0]) for t in tiles))
    same = ["=" if sums[r][k] == sums[-1][k] else "X" for k in range(len(sums[r]))]
    print(f"run {r:2d}: err {err:.1e}  last split per tile, per launch: {' | '.join(last)}  C tiles vs last run: "
          f"{''.join(same)}", flush=True)
