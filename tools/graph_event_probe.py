"""Probe: can timing events be recorded INSIDE a hipGraph so that every replay times the kernels
between them?  Tries the HIP paths one by one and prints their return codes and timings.

    python tools/graph_event_probe.py
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import sat_amd  # noqa: E402
from sat_amd import ops  # noqa: E402

dev = torch.device("cuda")
x = torch.randn(128, 14, 14, 256, device=dev).relu().bfloat16()
w = (torch.randn(256, 3, 3, 256, device=dev) * 0.03).bfloat16()
b = torch.zeros(256, device=dev)
f = (ops.mfma_frag_layout(w.reshape(256, -1)), b)
y = ops.conv3x3_frag(x, f)
torch.cuda.synchronize()
hip = ctypes.CDLL("libamdhip64.so.7")
vp = ctypes.c_void_p


def ev_new(flags=0):
    e = vp()
    rc = hip.hipEventCreateWithFlags(ctypes.byref(e), ctypes.c_uint(flags))
    assert rc == 0, rc
    return e


def elapsed(e0, e1):
    ms = ctypes.c_float()
    rc = hip.hipEventElapsedTime(ctypes.byref(ms), e0, e1)
    return ms.value * 1e3 if rc == 0 else f"rc={rc}"


n = 8
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
st.record()
for _ in range(n):
    ops.conv3x3_frag(x, f, out=y)
en.record()
en.synchronize()
print(f"eager back-to-back: {st.elapsed_time(en) / n * 1e3:.2f} us/launch", flush=True)

for label, flags in (("hipEventCreate default + record External", 0), ("blocking-sync event + External", 1)):
    evs = [(ev_new(flags), ev_new(flags)) for _ in range(n)]
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    codes = []
    try:
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                cs = vp(torch.cuda.current_stream().cuda_stream)
                for e0, e1 in evs:
                    codes.append(hip.hipEventRecordWithFlags(e0, cs, ctypes.c_uint(1)))
                    ops.conv3x3_frag(x, f, out=y)
                    codes.append(hip.hipEventRecordWithFlags(e1, cs, ctypes.c_uint(1)))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        print(f"{label}: record codes {sorted(set(codes))}; per-launch "
              f"{[elapsed(e0, e1) for e0, e1 in evs]}", flush=True)
    except Exception as exc:   # noqa: BLE001
        print(f"{label}: codes {sorted(set(codes))} -> {exc}", flush=True)
        torch.cuda.synchronize()

# explicit event-record nodes added to the captured graph before instantiation (keep_graph=True)
try:
    g = torch.cuda.CUDAGraph(keep_graph=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                ops.conv3x3_frag(x, f, out=y)
    graph = vp(g.raw_cuda_graph())
    cnt = ctypes.c_size_t(0)
    print("hipGraphGetNodes", hip.hipGraphGetNodes(graph, None, ctypes.byref(cnt)), cnt.value, flush=True)
    nodes = (vp * cnt.value)()
    print("hipGraphGetNodes", hip.hipGraphGetNodes(graph, nodes, ctypes.byref(cnt)), flush=True)
    e0, e1 = ev_new(0), ev_new(0)
    # e0 before everything (no dependencies), e1 after the last node
    n0, n1 = vp(), vp()
    print("add e0", hip.hipGraphAddEventRecordNode(ctypes.byref(n0), graph, None, ctypes.c_size_t(0), e0), flush=True)
    kinds = []
    for i in range(cnt.value):
        t = ctypes.c_int()
        hip.hipGraphNodeGetType(nodes[i], ctypes.byref(t))
        kinds.append(t.value)
    print("node types", kinds, flush=True)
    roots = [nodes[i] for i in range(cnt.value)]
    dep = (vp * 1)(n0)
    first = roots[0]
    print("dep e0->first", hip.hipGraphAddDependencies(graph, dep, (vp * 1)(first), ctypes.c_size_t(1)), flush=True)
    last = (vp * 1)(roots[-1])
    print("add e1", hip.hipGraphAddEventRecordNode(ctypes.byref(n1), graph, last, ctypes.c_size_t(1), e1), flush=True)
    g.instantiate()
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        print("explicit nodes: span of", n, "launches", elapsed(e0, e1), "us", flush=True)
except Exception as exc:   # noqa: BLE001
    print("explicit nodes:", exc, flush=True)
