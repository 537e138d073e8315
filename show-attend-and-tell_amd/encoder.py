"""Encoder module (reference: encoder.py:5-40) on MFMA implicit-GEMM convolutions.

``Encoder(network)`` keeps the reference attributes (``network``, ``net``,
``dim``) and the torchvision 0.16 parameter layout of ``self.net``
(``vgg19().features[:-1]`` -> keys ``net.<i>.weight``; ``resnet152`` children
``[:-2]`` -> ``net.0`` conv1, ``net.1`` bn1, ``net.4-7`` layer1-4 Bottlenecks), so
torchvision-derived state_dicts load unchanged.  ``forward(x[B,3,H,W]) ->
[B, L, D]`` runs the trunk as a compiled plan of HIP kernels on NHWC
activations:

  * every Conv2d (+ eval-mode BatchNorm folded into weight/bias, + ReLU, + the
    residual add of a Bottleneck) is ONE implicit-GEMM MFMA launch
    (sat_conv2d_nhwc): M = B*OH*OW, N = Cout, K = KH*KW*Cin;
  * MaxPool2d is a streaming NHWC kernel;
  * the image is converted once to NHWC with channels zero-padded 3 -> 8 so the
    first conv loads 16-byte vectors (VGG19); for ResNet152 it is converted to a
    2x2 space-to-depth layout instead ([H/2, W/2, 16], 12 real channels) and the
    7x7 / stride-2 / pad-3 stem runs as the equivalent 4x4 / stride-1 conv with
    re-laid-out weights (K = 256 instead of 7*7*8 = 392, half the input bytes);
  * the final NHWC tensor already IS ``permute(0,2,3,1).view(B,-1,C)``
    (encoder.py:37-39): no transpose.

The trunk is frozen (``requires_grad=False``) and forward-only for every
network: the reference freezes only VGG19 (encoder.py:29-31) and lets ResNet152
accumulate encoder gradients the optimiser never reads (train.py:71); skipping
that dead backward leaves every trained value identical.
Pretrained ImageNet weights are a download in the reference; here weights are
randomly initialised with torchvision's scheme unless a state_dict is loaded.
DenseNet161 (argparse choice, no BASELINE config) is out of scope.
"""
import torch
import torch.nn as nn

from . import _lib as L
from . import ops
from .data import PackedImages

VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]
IN_PAD = 8  # input channels padded 3 -> 8 (16-B bf16 vectors in the im2col loader)
S2D_C = 16  # space-to-depth stem input channels (2*2*3 real, zero-padded)


def stem_weight_s2d(w):
    """[Cout, KH=7, KW=7, Cin<=4] (NHWC-ordered, folded) stride-2 / pad-3 stem weights -> the
    [Cout, 4, 4, 16] weights of the same conv over the space-to-depth input: input row
    ih = 2*oh - 3 + kh = 2*(oh - 2 + th) + sy with kh + 1 = 2*th + sy, so tap (th, tw) and
    sub-pixel (sy, sx) of channel c land in s2d channel (sy*2 + sx)*Cin + c; the (kh + 1 = 0)
    row / column of the 8x8 footprint carries zero weight."""
    cout, kh_n, kw_n, cin = w.shape
    assert kh_n == 7 and kw_n == 7 and 4 * cin <= S2D_C
    out = torch.zeros(cout, 4, 4, S2D_C, dtype=w.dtype, device=w.device)
    for kh in range(7):
        th, sy = divmod(kh + 1, 2)
        for kw in range(7):
            tw, sx = divmod(kw + 1, 2)
            c0 = (sy * 2 + sx) * cin
            out[:, th, tw, c0:c0 + cin] = w[:, kh, kw, :]
    return out


class Bottleneck(nn.Module):
    """torchvision Bottleneck (expansion 4, stride on the 3x3: ResNet v1.5)."""
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride


def _vgg19_features():
    layers, cin = [], 3
    for v in VGG19_CFG:
        if v == "M":
            layers.append(nn.MaxPool2d(2, 2))
        else:
            layers += [nn.Conv2d(cin, v, 3, padding=1), nn.ReLU(inplace=True)]
            cin = v
    return layers[:-1]   # encoder.py:24-27 drops the last MaxPool


def _resnet152_trunk():
    layers = [nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
              nn.MaxPool2d(3, 2, 1)]
    inplanes = 64
    for li, (n, planes) in enumerate(zip([3, 8, 36, 3], [64, 128, 256, 512])):
        stride = 1 if li == 0 else 2
        blocks = []
        for bi in range(n):
            s = stride if bi == 0 else 1
            ds = None
            if bi == 0 and (s != 1 or inplanes != planes * 4):
                ds = nn.Sequential(nn.Conv2d(inplanes, planes * 4, 1, stride=s, bias=False), nn.BatchNorm2d(planes * 4))
            blocks.append(Bottleneck(inplanes, planes, s, ds))
            inplanes = planes * 4
        layers.append(nn.Sequential(*blocks))
    return layers


def _init_like_torchvision(module):
    """torchvision's init (kaiming-normal fan_out convs, BN gamma=1 beta=0), except that the
    last BN of every Bottleneck starts at gamma=0.2: with plain gamma=1 the 50 residual
    blocks double the activation variance per block (output std ~1e7 at random init),
    whereas a pretrained trunk -- which this random init stands in for -- emits O(1)
    features.  (torchvision's own zero_init_residual option uses gamma=0, which would feed
    the conv3 MFMAs all-zero weights and flatter their timing.)"""
    for m in module.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.BatchNorm2d):
            nn.init.constant_(m.weight, 1)
            nn.init.constant_(m.bias, 0)
    for m in module.modules():
        if isinstance(m, Bottleneck):
            nn.init.constant_(m.bn3.weight, 0.2)


class Encoder(nn.Module):
    def __init__(self, network="vgg19", dtype=torch.float32):
        super().__init__()
        self.network = network
        if network == "resnet152":
            self.net = nn.Sequential(*_resnet152_trunk())
            self.dim = 2048
        elif network == "densenet161":
            raise NotImplementedError("densenet161 is out of scope for the MI355X path (no BASELINE config)")
        else:
            self.net = nn.Sequential(*_vgg19_features())
            self.dim = 512
        _init_like_torchvision(self.net)
        for p in self.net.parameters():   # frozen trunk (encoder.py:29-31; see module docstring)
            p.requires_grad = False
        self.compute_dtype = dtype
        self._plan = None
        self._plan_key = None
        self.timing = None   # bench hook: list collecting (start, end) HIP events around every conv launch
        self.timing_args = None   # bench hook: list collecting every conv launch's arguments
        # (a fused bottleneck launch is recorded as ("fused", x, frags))
        # bench hook: callable() -> the SatPolicy of the next conv launch (bench.py gives every launch its own
        # in-kernel timestamp slots, SatPolicy.stamps); None = self.policy for every launch
        self.launch_policy = None
        # identity-residual bottlenecks the fused kernel supports run as ONE launch
        # (sat_bottleneck_fused, csrc/convblock.hip); False = three conv launches (A/B, tests);
        # an int n fuses every n-th eligible block only (the unfused ones leave CUs to a decoder
        # running beside the encoder: bench.py --fuse-every)
        self.fuse_blocks = True
        # layer2's identity bottlenecks (28 x 28, 512 -> 128) as ONE launch each (the band form of
        # sat_bottleneck_fused); independent of fuse_blocks, which governs the 14 x 14 layer3 blocks.  Off: at
        # B = 128 the fused band kernel is no faster than the three launches (112 vs 106 us; B = 64: 51 vs 60)
        # and its 159 KB of LDS per CU slow the overlapped train step (profiles/r3_s22)
        self.fuse_layer2 = False
        # the c2 of an identity block left unfused runs on the half-image conv kernel
        # (sat_conv3x3_frag: input rows staged once in LDS, fragment-layout weights); False = the
        # tile kernel (A/B, tests)
        self.c2_frag = True
        # ... at these spatial sizes (layer4 7, layer3 14, layer2 28; VGG19 block 5 14, block 2 112);
        # A/B: bench.py --c2-frag-sizes
        self.c2_frag_sizes = (7, 14, 28, 56, 112)
        # ... its c1 on the half-image 1x1 kernel (sat_conv1x1_frag: input slabs by LDS-DMA, weights
        # register-direct)
        self.c1_frag = True
        # per-call kernel selection for the conv launches (sat_amd.Policy / SatPolicy; None = the library's
        # defaults): A/B measurements and tests only
        self.policy = None

    def _launch(self, record, fn, *args, **kw):
        """One conv launch with the bench's hooks: its arguments recorded, an event pair around it,
        the in-graph launch timer's marks."""
        if self.timing_args is not None:
            self.timing_args.append(record)
        kw["policy"] = self.launch_policy() if self.launch_policy is not None else self.policy
        if self.timing is None:
            y = fn(*args, **kw)
        else:
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            y = fn(*args, **kw)
            en.record()
            self.timing.append((st, en))
        return y

    def _conv(self, x, f, relu, residual=None, out_hw=None):
        w, b, s, p = f
        return self._launch((x, w, b, s, p, relu, residual, out_hw), ops.conv2d_nhwc, x, w, b, s, p, relu,
                            residual=residual, out_hw=out_hw)

    def _frag_conv(self, kind, fn, x, f, *extra):
        """A half-image fragment-weight conv launch (csrc/convblock.hip), with the bench's hooks."""
        return self._launch((kind, x, f) + extra, fn, x, f, *extra)

    # ---- plan: folded NHWC weights ------------------------------------------
    @torch.no_grad()
    def _fold(self, conv, bn, pad_in=None):
        w = conv.weight.detach().float()
        b = conv.bias.detach().float() if conv.bias is not None else torch.zeros(w.shape[0], device=w.device)
        if bn is not None:  # eval-mode BatchNorm2d folded into the conv
            scale = bn.weight.float() / torch.sqrt(bn.running_var.float() + bn.eps)
            w = w * scale[:, None, None, None]
            b = bn.bias.float() + (b - bn.running_mean.float()) * scale
        w = w.permute(0, 2, 3, 1)   # [Cout, KH, KW, Cin]
        if pad_in is not None and w.shape[3] < pad_in:
            w = torch.nn.functional.pad(w, (0, pad_in - w.shape[3]))
        return (w.contiguous().to(self.compute_dtype), b.contiguous(), conv.stride[0], conv.padding[0])

    def _state_key(self, device, dtype):
        return (device, dtype, tuple(p._version for p in self.net.parameters()),
                tuple(b._version for b in self.net.buffers()))

    def _build_plan(self, device, dtype):
        self.compute_dtype = dtype
        plan = []
        mods = list(self.net.children())
        if self.network == "resnet152":
            w, b, _, _ = self._fold(mods[0], mods[1])
            plan.append(("stem_s2d", (stem_weight_s2d(w.float()).to(self.compute_dtype).contiguous(), b, 1, 2),
                         self._fold(mods[0], mods[1], IN_PAD)))
            plan.append(("pool", 3, 2, 1))
            for layer in mods[4:]:
                for blk in layer:
                    ds = self._fold(blk.downsample[0], blk.downsample[1]) if blk.downsample is not None else None
                    fused = self._fused_weights(plan, blk, ds)
                    plan.append(("block", self._fold(blk.conv1, blk.bn1), self._fold(blk.conv2, blk.bn2),
                                 self._fold(blk.conv3, blk.bn3), ds, fused,
                                 fused[1] if fused is not None else self._c2_frag_weights(blk)))
        else:
            first = True
            hw = 224   # spatial size at this conv for the 224 x 224 input the plan assumes (forward checks the real one)
            for i, m in enumerate(mods):
                if isinstance(m, nn.Conv2d):
                    relu = i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU)
                    f = self._fold(m, None, IN_PAD if first else None)
                    plan.append(("conv", f, relu, self._conv_frag_weights(m, f, relu, hw)))
                    first = False
                elif isinstance(m, nn.MaxPool2d):
                    plan.append(("pool", m.kernel_size, m.stride, m.padding))
                    hw //= 2
        self._plan = plan

    def _fused_weights(self, plan, blk, ds):
        """Fragment-layout weights of an identity-residual bottleneck the fused kernel runs, else None."""
        if ds is not None or blk.conv2.stride[0] != 1 or self.compute_dtype != torch.bfloat16 \
                or not blk.conv1.weight.is_cuda:
            return None
        # spatial size at this block: the trunk halves it at each stride-2 step (224 input assumed
        # by the plan; forward checks the activation's real size before taking the fused path)
        cin, cmid = blk.conv1.in_channels, blk.conv1.out_channels
        hw = {256: 56, 512: 28, 1024: 14, 2048: 7}.get(cin)
        if hw is None or not ops.bottleneck_fused_supported(hw, hw, cin, cmid, self.compute_dtype):
            return None
        frags = []
        for conv, bn in ((blk.conv1, blk.bn1), (blk.conv2, blk.bn2), (blk.conv3, blk.bn3)):
            w, b, _, _ = self._fold(conv, bn)
            frags.append((ops.mfma_frag_layout(w.reshape(w.shape[0], -1)), b))
        return tuple(frags)

    def _conv_frag_weights(self, conv, folded, relu, hw):
        """Fragment-layout weights of a VGG19 3x3 / stride-1 C -> C conv + ReLU that the staged-input kernel runs
        at its spatial size (sat_conv3x3_frag: the 14 x 14, 512 -> 512 block-5 convs), else None."""
        if not relu or conv.kernel_size != (3, 3) or conv.stride != (1, 1) or conv.padding != (1, 1) \
                or conv.in_channels != conv.out_channels or self.compute_dtype != torch.bfloat16 \
                or not conv.weight.is_cuda or not ops.conv3x3_frag_supported(hw, hw, conv.out_channels, self.compute_dtype):
            return None
        w, b = folded[0], folded[1]
        return ops.mfma_frag_layout(w.reshape(w.shape[0], -1)), b

    def _c2_frag_weights(self, blk):
        """Fragment-layout c2 weights of a stride-1 block whose 3x3 the band kernel runs (layer2), else None."""
        if blk.conv2.stride[0] != 1 or self.compute_dtype != torch.bfloat16 or not blk.conv2.weight.is_cuda:
            return None
        cmid = blk.conv2.out_channels
        hw = {64: 56, 128: 28, 256: 14, 512: 7}.get(cmid)
        if hw is None or not ops.conv3x3_frag_supported(hw, hw, cmid, self.compute_dtype):
            return None
        w, b, _, _ = self._fold(blk.conv2, blk.bn2)
        return ops.mfma_frag_layout(w.reshape(w.shape[0], -1)), b

    def compiled_plan(self, device, dtype):
        key = self._state_key(device, dtype)
        if self._plan is None or self._plan_key != key:
            self._build_plan(device, dtype)
            self._plan_key = key
        return self._plan

    def stage_starts(self, device=None, dtype=None):
        """Plan indices where each ResNet stage (layer1..layer4) starts; [] for VGG19."""
        plan = self.compiled_plan(device or next(self.parameters()).device, dtype or self.compute_dtype)
        starts, prev = [], None
        for i, step in enumerate(plan):
            if step[0] == "block":
                cout = step[3][0].shape[0]   # c3's output channels: 256 / 512 / 1024 / 2048
                if cout != prev:
                    starts.append(i)
                    prev = cout
        return starts

    def forward(self, x, dtype=None, steps=None):
        """Images [B,3,H,W] -> features [B, L, D].  ``steps=(start, stop)`` runs a slice of the
        plan (stage_starts()): start > 0 takes the NHWC activation the previous slice returned,
        stop < len(plan) returns the NHWC activation instead of [B, L, D]."""
        packed = isinstance(x, PackedImages)
        L.require_device(x.pixels if packed else x)
        dtype = dtype or self.compute_dtype
        plan = self.compiled_plan((x.pixels if packed else x).device, dtype)
        start, stop = steps if steps is not None else (0, len(plan))
        if packed:   # decoded uint8 images: resize + normalize straight into the first layer's layout
            if start > 0:
                raise ValueError("Encoder: packed images enter at plan step 0")
            if plan[0][0] == "stem_s2d":
                y = ops.images_to_input(x, L.IMG_S2D16, dtype)
                y = self._conv(y, plan[0][1], True, out_hw=(y.shape[1], y.shape[2]))
            else:
                y = ops.images_to_input(x, L.IMG_NHWC, dtype, c_pad=IN_PAD)
            return self._run_plan(y, plan, stop)
        if start > 0:
            y = x
            for step in plan[start:stop]:
                y = self._run_step(y, step)
            if stop < len(plan):
                return y
            B, H, W, C = y.shape
            return y.view(B, H * W, C)
        H, W = x.shape[2], x.shape[3]
        if plan[0][0] == "stem_s2d" and H % 2 == 0 and W % 2 == 0:
            y = ops.nchw_to_s2d(x, dtype)
            y = self._conv(y, plan[0][1], True, out_hw=(H // 2, W // 2))
        elif plan[0][0] == "stem_s2d":   # odd image sizes: the stem on the 8-channel layout
            y = self._conv(ops.nchw_to_nhwc(x, IN_PAD, dtype), plan[0][2], True)
        else:
            y = ops.nchw_to_nhwc(x, IN_PAD, dtype)
        return self._run_plan(y, plan, stop)

    @staticmethod
    def _block_cin(step):
        return step[1][0].shape[3]   # c1's folded weight [Cout, 1, 1, Cin]

    def _fuse_this(self, plan, step):
        if self._block_cin(step) == 512:
            return bool(self.fuse_layer2)
        f = self.fuse_blocks
        if f is True or f is False:
            return f
        elig = [s for s in plan if s[0] == "block" and s[5] is not None and self._block_cin(s) != 512]
        return next(i for i, s in enumerate(elig) if s is step) % int(f) == 0

    def _run_plan(self, y, plan, stop):
        for step in plan[:stop]:
            if step[0] == "stem_s2d":
                continue
            y = self._run_step(y, step)
        if stop < len(plan):
            return y
        B, H, W, C = y.shape
        return y.view(B, H * W, C)

    def _run_step(self, y, step):
        if step[0] == "conv":
            f = step[3]
            if f is not None and self.c2_frag and y.shape[1] in self.c2_frag_sizes \
                    and ops.conv3x3_frag_supported(y.shape[1], y.shape[2], y.shape[3], y.dtype):
                return self._frag_conv("c2frag", ops.conv3x3_frag, y, f)
            return self._conv(y, step[1], step[2])
        if step[0] == "pool":
            return ops.maxpool2d_nhwc(y, step[1], step[2], step[3])
        _, c1, c2, c3, ds, fused, c2f = step
        if (fused is not None and self._fuse_this(self._plan, step)
                and ops.bottleneck_fused_supported(y.shape[1], y.shape[2], y.shape[3], c1[0].shape[0], y.dtype)):
            return self._launch(("fused", y, fused), ops.bottleneck_fused, y, *fused)
        if fused is not None and self.c1_frag and ops.conv1x1_frag_supported(y.shape[1], y.shape[2], y.shape[3],
                                                                           c1[0].shape[0], y.dtype):
            out = self._frag_conv("c1frag", ops.conv1x1_frag, y, fused[0])
        else:
            out = self._conv(y, c1, True)
        if c2f is not None and self.c2_frag and out.shape[1] in self.c2_frag_sizes \
                and ops.conv3x3_frag_supported(out.shape[1], out.shape[2], out.shape[3],
                                                                         out.dtype):
            out = self._frag_conv("c2frag", ops.conv3x3_frag, out, c2f)
        else:
            out = self._conv(out, c2, True)
        idn = self._conv(y, ds, False) if ds is not None else y
        return self._conv(out, c3, True, residual=idn)
