"""Per-workgroup timeline of one conv launch (diagnostics build hook sat_fast_gemm_set_trace).

    python tools/conv_trace.py L3_c3 [tile] [stages]

Each workgroup records [start, main loop done, end, hw id] on the 100 MHz realtime clock.
Prints the launch span, per-workgroup main-loop / epilogue medians, workgroups per CU at once,
and the gap between a workgroup's end and the next start on the same CU.
"""
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import sat_amd  # noqa: E402
from sat_amd import ops  # noqa: E402
from conv_one import SHAPES  # noqa: E402  (tools/ on sys.path when run as a script)

name = sys.argv[1]
tile = int(sys.argv[2]) if len(sys.argv) > 2 else 0
stages = int(sys.argv[3]) if len(sys.argv) > 3 else 0
H, C, Co, k, s, p, r = SHAPES[name]
B = 128
x = torch.randn(B, H, H, C, device="cuda").bfloat16()
w = (torch.randn(Co, k, k, C, device="cuda") / (k * k * C) ** 0.5).bfloat16()
b = torch.randn(Co, device="cuda")
OH = (H + 2 * p - k) // s + 1
res = torch.randn(B, OH, OH, Co, device="cuda").bfloat16() if r else None
y = torch.empty(B, OH, OH, Co, device="cuda", dtype=torch.bfloat16)
lib = sat_amd._lib.lib()
lib.sat_fast_gemm_set_config(stages, tile, 1)
bm = 256 if tile == 5 else 128
bn = {2: 64, 4: 256}.get(tile, 128)
ntiles = max(-(-B * OH * OH // bm) * -(-Co // bn), 512)
buf = torch.zeros(ntiles * 4, dtype=torch.int64, device="cuda")
for _ in range(3):
    ops.conv2d_nhwc(x, w, b, s, p, True, residual=res, out=y)
torch.cuda.synchronize()
lib.sat_fast_gemm_set_trace(ctypes.c_void_p(buf.data_ptr()))
ops.conv2d_nhwc(x, w, b, s, p, True, residual=res, out=y)
torch.cuda.synchronize()
lib.sat_fast_gemm_set_trace(ctypes.c_void_p(0))
rec = [r_ for r_ in buf.view(ntiles, 4).cpu().tolist() if r_[0] != 0]
ntiles = len(rec)
t0 = min(r_[0] for r_ in rec)
span = (max(r_[2] for r_ in rec) - t0) * 0.01
main = [(r_[1] - r_[0]) * 0.01 for r_ in rec]
epi = [(r_[2] - r_[1]) * 0.01 for r_ in rec]
cus = {}
for r_ in rec:
    hw = r_[3] & 0xFFFFFFFF
    key = (r_[3] >> 32, (hw >> 8) & 0xFF)
    cus.setdefault(key, []).append(r_)
gaps, conc = [], []
for key, lst in cus.items():
    lst.sort()
    ends = sorted(q[2] for q in lst)
    # for each start after the first round, the gap to the latest end before it on this CU
    for q in lst:
        prev = [e for e in ends if e <= q[0]]
        if prev:
            gaps.append((q[0] - prev[-1]) * 0.01)
    # workgroups resident at each start
    for q in lst:
        conc.append(sum(1 for o in lst if o[0] <= q[0] < o[2]))
first_starts = sorted((r_[0] - t0) * 0.01 for r_ in rec)[:512]


def q(v):
    v = sorted(v)
    return f"p10 {v[len(v) // 10]:.2f}  p50 {statistics.median(v):.2f}  p90 {v[9 * len(v) // 10]:.2f}"


print(f"{name}: {ntiles} workgroups on {len(cus)} CUs, launch span {span:.1f} us")
print(f"  main loop us  {q(main)}")
print(f"  epilogue us   {q(epi)}")
print(f"  gap end->next start on a CU us  {q(gaps) if gaps else '-'}")
print(f"  resident workgroups per CU at a start  {q(conc)}")
print(f"  first 512 starts spread: {first_starts[0]:.2f} .. {first_starts[-1]:.2f} us")
per_cu = [len(v) for v in cus.values()]
print(f"  workgroups per CU: min {min(per_cu)} max {max(per_cu)}")
