"""Ablation of the layer3 c2 half-image kernel (conv3x3_frag_kernel, csrc/convblock.hip) at B = 128: the same launch
timed back to back with the product library and with diagnostics builds that drop one of its three streams
(SAT_C2_ABL bits: 1 no weight streaming, 2 no MFMA, 4 no A-fragment LDS reads; tools/build_c2_ablation.sh builds
show-attend-and-tell_amd/libsat_hip_abl<N>.so).  Each library runs in its own process (SAT_HIP_LIB_TUNING).

    python tools/c2_ablation.py            # parent: every library found
    python tools/c2_ablation.py --one      # child: the library SAT_HIP_LIB_TUNING names
"""
import glob
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def one(B=128, reps=50):
    import torch
    import sat_amd
    from sat_amd import ops
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    C = 256
    x = torch.randn(B, 14, 14, C, device=dev, generator=g).relu().bfloat16()
    w = (torch.randn(C, 3, 3, C, device=dev, generator=g) * (2.0 / (9 * C)) ** 0.5).bfloat16()
    f = (ops.mfma_frag_layout(w.reshape(C, 9 * C)), 0.1 * torch.randn(C, device=dev, generator=g))
    y = torch.empty_like(x)
    for _ in range(5):
        ops.conv3x3_frag(x, f, out=y)
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        ops.conv3x3_frag(x, f, out=y)
    en.record()
    en.synchronize()
    us = st.elapsed_time(en) * 1e3 / reps
    print(json.dumps({"lib": os.path.basename(os.environ.get("SAT_HIP_LIB_TUNING", "libsat_hip.so")), "us": round(us, 2),
                      "tflops": round(2.0 * B * 196 * C * 9 * C / us / 1e6, 1)}))


def main():
    libs = [None] + sorted(glob.glob(os.path.join(REPO, "show-attend-and-tell_amd", "libsat_hip_abl*.so")))
    for lib in libs:
        env = dict(os.environ)
        if lib:
            env["SAT_HIP_LIB_TUNING"] = lib
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--one"], env=env, capture_output=True, text=True,
                           timeout=120)
        print(r.stdout.strip() or r.stderr[-2000:], flush=True)


if __name__ == "__main__":
    one() if "--one" in sys.argv else main()
