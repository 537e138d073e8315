"""Probe (GPU): which HIP events can be recorded as event-record nodes inside a torch-captured graph, from
Python (ctypes) and from libsat_hip (SatPolicy.step_events through the decoder)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipEventRecordWithFlags.restype = ctypes.c_int
hip.hipEventRecordWithFlags.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
hip.hipGetLastError.restype = ctypes.c_int
vp = ctypes.c_void_p
x = torch.randn(1 << 20, device="cuda")


def new_event(flags):
    e = vp()
    rc = hip.hipEventCreateWithFlags(ctypes.byref(e), ctypes.c_uint(flags))
    return e if rc == 0 else None


for label in ("torch timing event", "hipEventCreateWithFlags(0)", "hipEventCreateWithFlags(2: disable timing)"):
    if label.startswith("torch"):
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for e in evs:
            e.record()
        handles = [vp(e.cuda_event) for e in evs]
    else:
        handles = [new_event(0 if "(0)" in label else 2) for _ in range(2)]
    torch.cuda.synchronize()
    print("outside capture:", label, [hip.hipEventRecordWithFlags(h, vp(torch.cuda.current_stream().cuda_stream), 1)
                                       for h in handles], "last", hip.hipGetLastError(), flush=True)
    g = torch.cuda.CUDAGraph()
    codes = []
    try:
        with torch.cuda.graph(g):
            cs = vp(torch.cuda.current_stream().cuda_stream)
            codes.append(hip.hipEventRecordWithFlags(handles[0], cs, 1))
            y = x * 2
            codes.append(hip.hipEventRecordWithFlags(handles[1], cs, 1))
        g.replay()
        torch.cuda.synchronize()
        ms = ctypes.c_float()
        rc = hip.hipEventElapsedTime(ctypes.byref(ms), handles[0], handles[1])
        print("in capture:", label, codes, "elapsed rc", rc, ms.value * 1e3, "us; last", hip.hipGetLastError(),
              flush=True)
    except Exception as exc:  # noqa: BLE001
        print("in capture:", label, codes, "->", exc, flush=True)
        torch.cuda.synchronize()
