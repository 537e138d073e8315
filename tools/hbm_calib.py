"""HBM calibration for the residual-conv traffic mix: torch elementwise kernels over the L1_c3
tensor sizes (bf16, B=128): copy (205 MB r + 205 MB w), add (410 r + 205 w)."""
import torch
n = 401408 * 256
x = torch.randn(n, device="cuda").bfloat16(); y = torch.randn(n, device="cuda").bfloat16()
z = torch.empty_like(x)
def t(f, nb, name):
    for _ in range(3): f()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(20): f()
    en.record(); torch.cuda.synchronize()
    us = st.elapsed_time(en) / 20 * 1e3
    print(f"{name}: {us:.1f} us, {nb / us / 1e6:.2f} TB/s", flush=True)
t(lambda: z.copy_(x), 4 * n, "copy bf16 205MB")
t(lambda: torch.add(x, y, out=z), 6 * n, "add bf16 (2r+1w)")
t(lambda: x.float().sum(), 2 * n, "read-only sum")
t(lambda: z.fill_(1.0), 2 * n, "write-only fill")
