"""Probe: do timing events recorded INSIDE a hipGraph capture (hipEventRecordWithFlags with
hipEventRecordExternal -> an event-record node) time the kernels between them on replay?

    python tools/graph_event_probe.py

Prints the eager per-launch time of a conv (event pair per launch), the same launches inside a
captured graph bracketed by external event nodes, and the graph's replay span.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import sat_amd  # noqa: E402
from sat_amd import ops  # noqa: E402
from bench import graph_event_record  # noqa: E402

dev = torch.device("cuda")
x = torch.randn(128, 14, 14, 256, device=dev).relu().bfloat16()
w = (torch.randn(256, 3, 3, 256, device=dev) * 0.03).bfloat16()
b = torch.zeros(256, device=dev)
f = (ops.mfma_frag_layout(w.reshape(256, -1)), b)
y = ops.conv3x3_frag(x, f)
torch.cuda.synchronize()

n = 20
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
st.record()
for _ in range(n):
    ops.conv3x3_frag(x, f, out=y)
en.record()
en.synchronize()
print(f"eager back-to-back: {st.elapsed_time(en) / n * 1e3:.2f} us/launch", flush=True)

evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
for e0, e1 in evs:   # create the HIP events outside the capture
    e0.record()
    e1.record()
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    with torch.cuda.graph(g, stream=s):
        for e0, e1 in evs:
            graph_event_record(e0)
            ops.conv3x3_frag(x, f, out=y)
            graph_event_record(e1)
torch.cuda.synchronize()
for rep in range(3):
    a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    z.record()
    torch.cuda.synchronize()
    per = [e0.elapsed_time(e1) * 1e3 for e0, e1 in evs]
    print(f"graph replay {rep}: span {a.elapsed_time(z) * 1e3:.1f} us, in-graph event pairs: "
          f"mean {sum(per) / n:.2f} us, min {min(per):.2f}, max {max(per):.2f}", flush=True)
