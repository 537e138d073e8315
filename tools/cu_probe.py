"""Map the runtime's CU-mask bits to hardware (XCC, SE, SH, CU): launch a spinning probe kernel on
streams masked to single bits / bit groups and record the HW_ID / XCC_ID of every workgroup."""
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sat_amd  # noqa: E402
from sat_amd import _lib as L  # noqa: E402


def decode(hw, xcc):
    return dict(xcc=xcc & 0xF, se=(hw >> 13) & 0x7, sh=(hw >> 12) & 1, cu=(hw >> 8) & 0xF)


def probe(stream, nblocks=2048, spin=20000):
    out = torch.zeros(2 * nblocks, dtype=torch.int32, device="cuda")
    with torch.cuda.stream(stream):
        L.check(L.lib().sat_probe_cu_ids(nblocks, spin, L.ptr(out), ctypes_stream(stream)), "probe")
    torch.cuda.synchronize()
    o = out.cpu().tolist()
    return collections.Counter(tuple(sorted(decode(o[2 * i] & 0xFFFFFFFF, o[2 * i + 1]).items())) for i in range(nblocks))


def ctypes_stream(s):
    import ctypes
    return ctypes.c_void_p(s.cuda_stream)


def main():
    ncu = sat_amd.ops.device_cu_count()
    res = {"ncu": ncu}
    full = probe(torch.cuda.current_stream())
    res["full_distinct_cus"] = len(full)
    res["full_xcc_counts"] = dict(collections.Counter(dict(k)["xcc"] for k in full))
    single = {}
    for b in list(range(0, 64)) + [64, 96, 128, 160, 192, 224, 255]:
        s = sat_amd.ops.cu_masked_stream([b])
        c = probe(s, nblocks=64, spin=2000)
        single[b] = [dict(k) for k in c]
    res["single_bit"] = single
    for name, cus in (("first32", list(range(32))), ("every8", list(range(0, 256, 8)))):
        c = probe(sat_amd.ops.cu_masked_stream(cus))
        res[name] = {"distinct": len(c), "xcc": dict(collections.Counter(dict(k)["xcc"] for k in c)),
                     "se": dict(collections.Counter((dict(k)["xcc"], dict(k)["se"]) for k in c).most_common(8))}
    print(json.dumps(res, default=str))


if __name__ == "__main__":
    main()
