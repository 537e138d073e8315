"""Per-class conv time of the ResNet152 / VGG19 trunk (B=128, bf16) with the new conv kernels toggled:
stream (convstream.hip), pipe (convpipe.hip), halo (convhalo.hip) on/off, interleaved in one process.
    python tools/trunk_ab.py [network]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import sat_amd  # noqa: E402
import bench  # noqa: E402

net = sys.argv[1] if len(sys.argv) > 1 else "resnet152"
B = 128
lib = sat_amd._lib.lib()
torch.manual_seed(0)
enc = sat_amd.Encoder(net, dtype=torch.bfloat16).cuda().eval()
imgs = torch.randn(B, 3, 224, 224, device="cuda")
launches = bench.conv_launches(net, B, fused=enc.fuse_blocks)
MODES = [(1, 1, 1), (1, 1, 0), (0, 1, 1), (0, 0, 0)]   # (stream, pipe, halo)
res = {}
for rnd in range(2):
    for sm, pm, hm in MODES:
        lib.sat_conv_stream_set_mode(sm)
        lib.sat_conv_pipe_set_mode(pm)
        lib.sat_conv_halo_set_mode(hm)
        with torch.no_grad():
            enc(imgs)
        torch.cuda.synchronize()
        _, trunk = bench.trunk_roofline(enc, imgs, launches)
        res.setdefault((sm, pm, hm), []).append(trunk)
lib.sat_conv_stream_set_mode(1)
lib.sat_conv_pipe_set_mode(1)
lib.sat_conv_halo_set_mode(1)
classes = list(res[MODES[0]][-1]["classes"])
print(f"{'class':32s}" + "".join(f"  s{sm}p{pm}h{hm:<4d}" for sm, pm, hm in MODES))
for c in classes:
    print(f"{c:32s}" + "".join(f"  {min(t['classes'][c]['us'] for t in res[m]):9.1f}" for m in MODES))
print(f"{'total':32s}" + "".join(f"  {min(t['conv_us_per_forward'] for t in res[m]):9.1f}" for m in MODES))
