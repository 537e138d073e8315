"""Benchmark: train images/sec of the Show-Attend-and-Tell step on MI355X.

Workload (BASELINE.json metric "train images/sec on COCO batch=128 at 1/2/4/8 MI355X"):
COCO-shaped synthetic batches -- 128 images/GPU of 224x224 (weak scaling), ResNet152
encoder (bf16, forward), decoder with --attention --tf --ado (E=512, D=2048, L=49),
V=10000, T=27 caption slots; random-init weights (no checkpoints offline).
One step = encoder fwd + decoder fwd + fused loss + decoder bwd + RCCL grad
all-reduce (N>1) + Adam, inputs resident in HBM before the timed region.

Run:  python bench.py [--gpus N --steps K --warmup W]
      N > 1: this process starts the N rank processes itself (torch.distributed.run, one rank per GPU, before
      anything touches a GPU) and exits with their status; launched by torch.distributed.run directly it is one
      of the ranks (WORLD_SIZE set) and checks that WORLD_SIZE == --gpus.
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BF16_DENSE_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: ~2.5 PF dense bf16 MFMA
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=128, help="images per GPU")
    ap.add_argument("--network", default="resnet152", choices=["resnet152", "vgg19"])
    ap.add_argument("--vocab", type=int, default=10000)
    ap.add_argument("--seq", type=int, default=27)
    ap.add_argument("--no-tf", action="store_true",
                    help="cfg4: no teacher forcing (greedy argmax feedback inside the time loop, decoder.py:131-133)")
    ap.add_argument("--bert", action="store_true",
                    help="cfg5: frozen BERT word embeddings (V=30522, E=768, T=32), simple deep output (--ado off)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=8,
                    help="images per step of the bounded CPU-baseline sample (the reference's cfg1 batch)")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraph replay")
    ap.add_argument("--no-overlap", action="store_true",
                    help="graph mode: run the next batch's encoder after, not beside, this batch's decoder")
    ap.add_argument("--feature-buffers", type=int, default=3, choices=[2, 3, 4],
                    help="graph + overlap: encoder output buffers (and graph sets) in flight; the next batch's encoder waits "
                         "for the decoder that last read its buffer (3: B = 64 4.08-4.11 vs 4.15 ms with 2, B = 128 "
                         "within noise; profiles/r3_s31)")
    ap.add_argument("--split-target", type=int, default=None,
                    help="graph + overlap: workgroups the decoder's per-step split-K GEMMs aim for (default: "
                         "64 with ResNet152 features, 128 with VGG19's: profiles/r2_s54_sched.txt)")
    ap.add_argument("--no-fuse-blocks", action="store_true",
                    help="run the layer3 identity bottlenecks as three conv launches (A/B of csrc/convblock.hip)")
    ap.add_argument("--bwd", choices=["auto", "serial", "split"], default="auto",
                    help="N = 1 decoder backward structure: one graph in order (serial), or two graphs as at N > 1 "
                         "(split: the head bucket's all-reduce runs between them); auto = serial at N = 1 (6.43-6.46 "
                         "vs 6.48-6.54 ms split, profiles/r3_s51), split at N > 1")
    ap.add_argument("--no-transposed", action="store_true",
                    help="BPTT input-gradient products on the k-major weights instead of the transposed copies (A/B)")
    ap.add_argument("--no-skinny", action="store_true",
                    help="per-step decoder GEMMs on the LDS-DMA tile kernel instead of csrc/skinny.hip (A/B)")
    ap.add_argument("--dp-rehearse", action="store_true",
                    help="N = 1 only: run the data-parallel path anyway (a one-rank process group over --dist-backend: "
                         "the eager warm-up's bucket all-reduces, the graphs captured beside the live watchdog, the "
                         "async bucket all-reduces between replays) -- the RCCL code of the N > 1 runs on a one-GPU box")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="N > 1: RCCL (one rank per GPU) or gloo (rehearsal: several ranks may share a GPU)")
    ap.add_argument("--gemm-stages", type=int, default=0, choices=[0, 2, 3],
                    help="LDS ring depth of the bf16 tile GEMM kernel (0 = auto: 3 for the decoder's per-step "
                         "split-K GEMMs, 2 otherwise)")
    ap.add_argument("--no-ws3x3", action="store_true",
                    help="64 -> 64 3x3 convs on the implicit-GEMM tile kernel instead of csrc/conv3x3ws.hip (A/B)")
    ap.add_argument("--conv-slices", type=int, default=0, choices=[0, 1, 2],
                    help="layer3 c1 / c2 kernels: 0 auto (two 128-channel slices per half image at B <= 64), 1 one "
                         "workgroup per half image, 2 two slices (SatPolicy.conv_slices, A/B)")
    ap.add_argument("--policy", default="",
                    help="extra SatPolicy fields for every encoder / decoder call, e.g. attn_bwd_chunks=1,gemm_stages=3 "
                         "or decoder_splits=2.0.0.0 (A/B; include/sat_hip.h)")
    ap.add_argument("--c2-frag-sizes", default="7,14,28,56,112",
                    help="spatial sizes whose stride-1 3x3 convs run on the staged-input kernels (sat_conv3x3_frag); "
                         "the others on the tile kernel (A/B)")
    ap.add_argument("--fuse-layer2", action="store_true",
                    help="layer2's identity bottlenecks as one fused band-kernel launch each instead of three conv "
                         "launches (A/B: profiles/r3_s22)")
    ap.add_argument("--fuse-every", type=int, default=None,
                    help="fuse every n-th layer3 identity bottleneck only, the rest run as three conv launches "
                         "(default 0 = none: with the layer3 c2 / c3 on the half-image frag kernels the unfused "
                         "trunk shares CUs with the decoder best; profiles/r2_s62_sched.txt)")
    ap.add_argument("--stream-priority", choices=["decoder-high", "equal", "encoder-high"], default="decoder-high",
                    help="graph + overlap: the decoder / all-reduce / Adam stream gets the higher HIP stream "
                         "priority, so its short per-step kernels are dispatched first when CUs free up")
    ap.add_argument("--fp32-steps", type=int, default=3,
                    help="timed steps of the fp32 leg (the reference's precision, the exact-parity path; 0 = skip)")
    ap.add_argument("--no-diagnostics", action="store_true",
                    help="skip the per-kernel roofline measurements after the timed region")
    ap.add_argument("--no-step-stamps", action="store_true",
                    help="graph mode: no stamped diagnostic copies of the graphs after the timed region (the in-step "
                         "conv / decoder figures, LaunchStamps / DecoderStamps; the timed graphs never carry stamps)")
    args = ap.parse_args()
    if args.bert:   # generate_json_data_bert.py:47,69: [CLS] + 30 + [SEP]; BertConfig() vocabulary
        args.vocab = 30522
        if args.seq == 27:
            args.seq = 32
        args.no_cpu_baseline = True   # the oracle's CPU-baseline sample covers the plain-vocab decoder only
    return args


PEAK_HBM_ACHIEVABLE_GBS = 6300.0   # MI355X_MICROARCH.md §HBM (floor estimates only)

class LaunchStamps:
    """In-kernel launch timestamps for a sequence of launches (SatPolicy.stamps): a device buffer of
    ``cap`` workgroup slots {start, end} per launch, and one SatPolicy per launch pointing at its slice.
    Every workgroup of a launch records when its first wave started and its last wave finished (the
    device's 100 MHz real-time counter); the launch's span is max(end) - min(start) -- the kernel's own
    duration inside the overlapped graph replays, with no extra node, event or barrier in the stream.
    The slots' enable words are off during the timed region (a launch then pays one scalar load) and on
    for a diagnostic phase of the same overlapped schedule right after it, and for replays of each graph on
    its own.  Timing events cannot be captured as graph nodes on this runtime (hipEventRecordWithFlags(..,
    hipEventRecordExternal) returns hipErrorInvalidValue during capture: tools/event_node_probe.py,
    profiles/r3_s9/probe.log), and a rocprofv3 kernel trace all but serialises the two streams (2.6 % of the
    traced busy time had kernels of two queues running, profiles/r3_s8/prof_summary.json) and adds its own
    per-dispatch signalling to every duration, so neither gives in-step kernel durations."""

    def __init__(self, n_launches, device, base=None, cap=16384):
        import sat_amd
        self.n, self.cap = n_launches, cap
        # per launch: a 16-B header (enable word) + cap workgroup records (SatPolicy.stamps)
        self.buf = torch.zeros(n_launches, cap + 1, 2, dtype=torch.int64, device=device)
        self.pols = []
        for k in range(n_launches):
            pol = sat_amd.Policy()
            if base is not None:
                __import__("ctypes").pointer(pol)[0] = base
            pol.stamps = self.buf[k].data_ptr()
            pol.stamp_capacity = cap
            self.pols.append(pol)
        self.used = 0

    def next_policy(self):
        if self.used >= self.n:
            raise RuntimeError("LaunchStamps: more launches than slots")
        self.used += 1
        return self.pols[self.used - 1]

    def enable(self, on):
        """Switch the launches' timestamps on / off (their enable words; graph replays read them)."""
        self.buf[:, 0, 0] = 1 if on else 0
        if on:
            self.buf[:, 1:].zero_()

    def spans_us(self):
        """Per launch (in launch order): max(end) - min(start) over its workgroups, microseconds."""
        st, en = self.buf[:self.used, 1:, 0], self.buf[:self.used, 1:, 1]
        valid = st > 0
        big = torch.iinfo(torch.int64).max
        lo = torch.where(valid, st, torch.full_like(st, big)).min(dim=1).values
        hi = torch.where(valid, en, torch.zeros_like(en)).max(dim=1).values
        return [((h - l) / 100.0 if h > 0 else None) for l, h in zip(lo.tolist(), hi.tolist())]   # 100 MHz ticks

    def intervals_us(self):
        """Per launch: first start of the NEXT launch minus its own first start (its span plus the boundary after
        it -- the launch's share of the stream), microseconds; None for the last launch."""
        st = self.buf[:self.used, 1:, 0]
        big = torch.iinfo(torch.int64).max
        lo = torch.where(st > 0, st, torch.full_like(st, big)).min(dim=1).values.tolist()
        return [((lo[i + 1] - lo[i]) / 100.0 if lo[i] < big and lo[i + 1] < big else None) for i in range(len(lo) - 1)] \
            + [None]


class DecoderStamps:
    """In-kernel timestamps of the decoder's per-step kernel groups (SatPolicy.stamps through
    SatDecoderDims.policy): the library gives group g (diagnostics.GROUPS order) at step t the slot
    g * (T-1) + t of ``cap`` workgroups; captured into the decoder graphs, every replay rewrites them."""

    def __init__(self, T, device, base=None, cap=1024):
        import sat_amd
        from sat_amd.diagnostics import GROUPS
        self.groups, self.T1, self.cap = GROUPS, T - 1, cap
        # slot g * (T-1) + t: a 16-B header (enable word) + cap workgroup records (decoder.hip step_slot)
        self.buf = torch.zeros(len(GROUPS) * self.T1, cap + 1, 2, dtype=torch.int64, device=device)
        self.policy = sat_amd.Policy()
        if base is not None:
            __import__("ctypes").pointer(self.policy)[0] = base
        self.policy.stamps = self.buf.data_ptr()
        self.policy.stamp_capacity = cap

    def enable(self, on):
        self.buf[:, 0, 0] = 1 if on else 0
        if on:
            self.buf[:, 1:].zero_()

    def _lo_hi(self):
        st, en = self.buf[:, 1:, 0], self.buf[:, 1:, 1]
        valid = st > 0
        big = torch.iinfo(torch.int64).max
        lo = torch.where(valid, st, torch.full_like(st, big)).min(dim=1).values.tolist()
        hi = torch.where(valid, en, torch.zeros_like(en)).max(dim=1).values.tolist()
        return lo, hi

    def chain_us(self):
        """Per time step of the forward (h_gemm .. lstm_fwd) and of the BPTT (lstm_bwd .. dh_gemm): the mean
        interval from one step's first kernel start to the next step's, beside the mean sum of the step's kernel
        spans -- the difference is what the dependent launches cost between kernels."""
        lo, hi = self._lo_hi()
        T1, gi = self.T1, {g: i for i, g in enumerate(self.groups)}

        def span(g, t):
            k = gi[g] * T1 + t
            return (hi[k] - lo[k]) / 100.0 if hi[k] > 0 else None

        def start(g, t):
            k = gi[g] * T1 + t
            return lo[k] if hi[k] > 0 else None
        out = {}
        for name, groups, order in (("fwd", self.groups[:4], range(T1)), ("bwd", self.groups[4:], range(T1 - 1, -1, -1))):
            order = list(order)
            iv, ks = [], []
            for a, b in zip(order, order[1:]):
                # the step's first launch to the next step's first launch; the spans of the groups the build runs
                # per step (groups folded into another kernel have no stamps)
                sa = next((start(g, a) for g in groups if start(g, a) is not None), None)
                sb = next((start(g, b) for g in groups if start(g, b) is not None), None)
                spans = [v for v in (span(g, a) for g in groups) if v is not None]
                if sa is not None and sb is not None and spans:
                    iv.append((sb - sa) / 100.0)
                    ks.append(sum(spans))
            if iv:
                out[f"{name}_step_interval_us"] = round(sum(iv) / len(iv), 2)
                out[f"{name}_step_kernels_us"] = round(sum(ks) / len(ks), 2)
        return out

    def group_spans_us(self):
        lo, hi = self._lo_hi()
        out = {}
        for gi, g in enumerate(self.groups):
            v = [(hi[k] - lo[k]) / 100.0 for k in range(gi * self.T1, (gi + 1) * self.T1) if hi[k] > 0]
            if v:
                out[g] = v
        return out

    def group_intervals_us(self):
        """Per group: first start of each of its launches to the first start of the next per-step launch of the
        chain (forward: steps 0 .. T-2, backward: T-2 .. 0, groups in launch order; groups a build no longer
        launches have no stamps and drop out) -- span plus the boundary after it, the per-dispatch duration a
        rocprofv3 kernel trace reports.  The last launch of each chain has no successor and no interval."""
        lo, hi = self._lo_hi()
        T1, ng = self.T1, len(self.groups)
        out = {}
        for order, gs in ((range(T1), range(0, ng // 2)), (range(T1 - 1, -1, -1), range(ng // 2, ng))):
            seq = [(g, t) for t in order for g in gs if hi[g * T1 + t] > 0]
            for (g, t), (g2, t2) in zip(seq, seq[1:]):
                out.setdefault(self.groups[g], []).append((lo[g2 * T1 + t2] - lo[g * T1 + t]) / 100.0)
        return out


def conv_launches(network, B, H=224, fused=True, fused2=False):
    """Every conv launch of one encoder forward, in launch order (encoder.py forward: per
    bottleneck c1, c2, downsample, c3, or ONE fused launch for the identity blocks the fused
    bottleneck kernel runs), with its algorithmic work: FLOPs = 2*M*N*K (real Cin=3 for the first
    conv) and bytes = input activation read once + weights + output (+ residual), bf16; a fused
    block reads its input once (the residual is the same tensor), writes its output once and reads
    its three weights.  ``bound`` is the roofline that is larger at 2.5 PFLOP/s / 6.3 TB/s."""
    out = []

    def bound_of(f, by):
        return "mfma" if f / (BF16_DENSE_PEAK_TFLOPS * 1e12) > by / (PEAK_HBM_ACHIEVABLE_GBS * 1e9) else "hbm"

    def add(name, M, N, K, in_elems, res=False, real_k=None):
        f = 2.0 * M * N * (real_k or K)
        by = 2.0 * (in_elems + N * K + M * N * (2 if res else 1))
        out.append(dict(cls=f"{name} {M}x{N}x{K}", flops=f, bytes=by, bound=bound_of(f, by)))

    def add_block(name, M, cin, pl):
        f = 2.0 * M * (cin * pl + 9 * pl * pl + pl * cin)
        by = 2.0 * (2 * M * cin + 2 * cin * pl + 9 * pl * pl)
        out.append(dict(cls=f"{name} {M}x{cin}x{pl}", flops=f, bytes=by, bound=bound_of(f, by), fused=True))

    if network == "resnet152":
        h = H // 2   # stem: 4x4 conv over the 2x2 space-to-depth input (16 channels, 12 real)
        add("stem7x7s2", B * h * h, 64, 4 * 4 * 16, B * h * h * 16, real_k=147)
        h //= 2
        cin = 64
        for li, (n, pl) in enumerate(zip([3, 8, 36, 3], [64, 128, 256, 512])):
            for bi in range(n):
                s = (1 if li == 0 else 2) if bi == 0 else 1
                oh = h // s
                if fused and bi > 0 and (h, cin, pl) == (14, 1024, 256) \
                        and (fused is True or (bi - 1) % int(fused) == 0):   # sat_bottleneck_fused_supported
                    add_block(f"L{li + 1}block(fused)", B * h * h, cin, pl)
                    continue
                if fused2 and bi > 0 and (h, cin, pl) == (28, 512, 128):   # layer2's band form
                    add_block(f"L{li + 1}block(fused)", B * h * h, cin, pl)
                    continue
                add(f"L{li + 1}c1", B * h * h, pl, cin, B * h * h * cin)
                add(f"L{li + 1}c2{'s2' if s == 2 else ''}", B * oh * oh, pl, 9 * pl, B * h * h * pl)
                if bi == 0:
                    add(f"L{li + 1}ds{'s2' if s == 2 else ''}", B * oh * oh, 4 * pl, cin, B * h * h * cin)
                add(f"L{li + 1}c3+res", B * oh * oh, 4 * pl, pl, B * oh * oh * pl, res=True)
                cin, h = 4 * pl, oh
    else:   # vgg19 features[:-1]: 16 3x3 convs, 4 pools (encoder.py:23-27)
        h, cin = H, 8
        for i, co in enumerate([64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M",
                                512, 512, 512, 512, "M", 512, 512, 512, 512]):
            if co == "M":
                h //= 2
                continue
            add(f"conv{i}", B * h * h, co, 9 * cin, B * h * h * cin, real_k=27 if cin == 8 else None)
            cin = co
    return out


def instep_conv_durations(stamps, launches, intervals=False):
    """Per conv launch (conv_launches() order), its in-step durations [us] from the encoder graphs'
    in-kernel timestamps (LaunchStamps, the last replay of each graph); intervals: launch-start to next
    launch-start instead of the span."""
    per = [[] for _ in launches]
    for st in stamps:
        spans = st.intervals_us() if intervals else st.spans_us()
        if len(spans) != len(launches):
            return None
        for i, us in enumerate(spans):
            if us is not None:
                per[i].append(us)
    return per


def trunk_roofline(enc, imgs, launches, instep=None, overlapped=None, intervals=None, reps=3):
    """The encoder trunk against its roofline.

    Per conv launch, up to three durations [us]:
      ``us``            the kernel's own first-start / last-end in-kernel timestamps in the captured encoder
                        graphs replayed on their own after the timed region (LaunchStamps, ``instep``);
      ``us_overlapped`` the same timestamps inside the timed region's overlapped schedule (``overlapped``);
      ``us_eager``      an event pair around every launch of ``reps`` eager forwards.
    The dominant class (largest per-forward time) and its ``achieved`` / ``frac`` come from ``us``; the others
    are reported beside it, with the class's launches re-issued back to back into warm caches
    (``avg_launch_us_b2b``).  A rocprofv3 kernel trace of the same command reports ~4 us more per conv
    dispatch: its per-dispatch completion signalling (profiles/r3_s8/prof_summary.json: under the trace these
    timestamps read 27.0 us for L3c2 where the trace reads 30.9 for the same launches)."""
    enc.timing, enc.timing_args = [], []
    with torch.no_grad():
        for _ in range(reps):
            enc(imgs)
    torch.cuda.synchronize()
    ev, enc.timing = enc.timing, None
    conv_args, enc.timing_args = enc.timing_args, None
    n = len(launches)
    assert len(ev) == reps * n, (len(ev), n)
    eager = [0.0] * n
    for r in range(reps):
        for i in range(n):
            st, en = ev[r * n + i]
            eager[i] += st.elapsed_time(en) / reps * 1e3   # us

    def mean_or_none(v):
        return [sum(x) / len(x) if x else None for x in v] if v is not None else [None] * n
    span, ov, itv = mean_or_none(instep), mean_or_none(overlapped), mean_or_none(intervals)
    primary = [s_ if s_ is not None else e for s_, e in zip(span, eager)]
    series = {"us": primary, "us_overlapped": ov, "us_eager": eager, "us_interval": itv}
    cls = {}
    for i, l in enumerate(launches):
        c = cls.setdefault(l["cls"], dict(n=0, flops=l["flops"], bytes=l["bytes"], bound=l["bound"],
                                          fused=l.get("fused", False), **{k: 0.0 for k in series}))
        c["n"] += 1
        for k, v in series.items():
            c[k] += v[i] if v[i] is not None else float("nan")
    name, dom = max(cls.items(), key=lambda kv: kv[1]["us"])
    idx = [i for i, l in enumerate(launches) if l["cls"] == name]
    # the dominant class's launches of the last forward re-issued back to back (same inputs, 5 each)
    from sat_amd import ops
    last = conv_args[(reps - 1) * n:]
    b2b = 5

    def launch(a):
        if a[0] == "fused":
            ops.bottleneck_fused(a[1], *a[2])
        elif a[0] == "c2frag":
            ops.conv3x3_frag(a[1], a[2])
        elif a[0] == "c1frag":
            ops.conv1x1_frag(a[1], a[2])
        else:
            x, w, b, s, p, relu, res, hw = a
            ops.conv2d_nhwc(x, w, b, s, p, relu, residual=res, out_hw=hw, policy=enc.policy)

    with torch.no_grad():
        for i in idx[:2]:   # warm
            launch(last[i])
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for i in idx:
            for _ in range(b2b):
                launch(last[i])
        en.record()
    en.synchronize()
    b2b_us = st.elapsed_time(en) / (len(idx) * b2b) * 1e3

    def rate(us):
        if dom["bound"] == "hbm":
            return dom["bytes"] / (us * 1e-6) / 1e9, HBM_PEAK_GBS, "GB/s"
        return dom["flops"] / (us * 1e-6) / 1e12, BF16_DENSE_PEAK_TFLOPS, "TFLOP/s"
    # the headline duration is the launch interval (start of the launch to start of the next one, graphs replayed
    # alone): the figure a rocprofv3 kernel trace of this command reproduces (its per-dispatch durations include the
    # same boundary); the kernel's own span is kept beside it as avg_launch_us_span / frac_span
    span_us = dom["us"] / dom["n"]
    itv_us = dom["us_interval"] / dom["n"]
    avg_us = itv_us if itv_us == itv_us else span_us
    achieved, peak, unit = rate(avg_us)
    extra = {"duration": "interval" if itv_us == itv_us else "span",
             "avg_launch_us_span": round(span_us, 2), "frac_span": round(rate(span_us)[0] / peak, 4)}
    for key, k in (("overlapped", "us_overlapped"),):
        a = dom[k] / dom["n"]
        if a == a:
            extra[f"avg_launch_us_{key}"] = round(a, 2)
            extra[f"frac_{key}"] = round(rate(a)[0] / peak, 4)
    floor_us = sum(max(l["flops"] / (BF16_DENSE_PEAK_TFLOPS * 1e12), l["bytes"] / (PEAK_HBM_ACHIEVABLE_GBS * 1e9))
                   for l in launches) * 1e6
    kname = "bottleneck_kernel (csrc/convblock.hip), fused block" if dom.get("fused") else (
        "conv3x3_frag_kernel (csrc/convblock.hip), conv class" if all(last[i][0] == "c2frag" for i in idx)
        else "conv1x1_frag_kernel (csrc/convblock.hip), conv class" if all(last[i][0] == "c1frag" for i in idx)
        else "conv kernels, conv class")
    timing = ("avg_launch_us (frac, achieved): first start of each launch of the class to the first start of the next "
              "launch, from in-kernel timestamps (LaunchStamps) in stamped copies of the encoder graphs replayed on "
              "their own after the timed region -- the kernel's span plus the boundary after it, the figure a "
              "rocprofv3 kernel trace of this command reproduces (profiles/<round>/prof_summary.json "
              "bench_over_rocprof); avg_launch_us_span / frac_span: the kernels' own first-start / last-end span; "
              "avg_launch_us_overlapped: the span inside the overlapped schedule (sharing CUs with the decoder "
              "graphs); avg_launch_us_b2b: the class re-issued back to back into warm caches; "
              f"avg_launch_us_eager_event_pairs: an event pair around every launch of {reps} eager forwards"
              if instep is not None else
              "avg_launch_us: an event pair around every launch of the eager forwards (no in-kernel timestamps)")

    def tot(k):
        v = sum(x for x in series[k] if x is not None) if any(x is not None for x in series[k]) else None
        return round(v, 1) if v is not None else None
    return dict(kernel=f"{kname} {name} ({dom['n']} launches/forward)", cls=name,
                bound=dom["bound"], achieved=round(achieved, 2), peak=peak, unit=unit,
                frac=round(achieved / peak, 4), avg_launch_us=round(avg_us, 2), **extra,
                avg_launch_us_b2b=round(b2b_us, 2), frac_b2b=round(rate(b2b_us)[0] / peak, 4),
                avg_launch_us_eager_event_pairs=round(dom["us_eager"] / dom["n"], 2),
                timing=timing, algorithmic_bytes_per_launch=dom["bytes"], algorithmic_flops_per_launch=dom["flops"]), \
        dict(conv_us_per_forward=tot("us"), conv_us_per_forward_overlapped=tot("us_overlapped"),
             conv_us_per_forward_eager=tot("us_eager"),
             roofline_floor_us=round(floor_us, 1), frac_of_floor=round(floor_us / tot("us"), 4),
             timing="per class: us = in-kernel timestamps (the encoder graphs replayed alone), us_overlapped = the "
                    "same in the timed region's overlapped schedule, us_eager = eager event pairs (roofline.timing)",
             classes={k: dict(n=v["n"], **{s_: round(v[s_], 1) for s_ in series if v[s_] == v[s_]})
                      for k, v in sorted(cls.items(), key=lambda kv: -kv[1]["us"])})


def pmc_traffic(network, cls):
    """HBM bytes per launch of conv class `cls` from the committed PMC passes
    (tools/pmc_traffic.py; a PMC run cannot share a process with the timed bench), else None."""
    path = os.path.join(REPO, "profiles", f"pmc_traffic_{network}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        rec = json.load(f)
    per = rec.get("classes", {}).get(cls)
    return (per["hbm_bytes_per_launch"] if per else None), os.path.relpath(path, REPO)


def usable_cores():
    """(cores this process may run on, cores of the host): the affinity mask capped by a cgroup CPU
    quota (a GPU box shares its host: os.cpu_count() reports the whole machine)."""
    host = os.cpu_count() or 1
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else host
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(math.ceil(int(quota) / int(period)))))
    except (OSError, ValueError):
        pass
    return n, host


def cpu_baseline(args):
    """Bounded CPU sample of the same train step through the oracle (torch-CPU fp32 port of the
    reference, oracle/sat_oracle.py), on every core this process may use, at --cpu-sample images per
    step (the reference's own cfg1 batch is 8).  Two variants, each ~8-15 s of host work:
    the frozen trunk (result-identical; the headline CPU number) and the reference as it runs,
    whose ResNet152 parameters are not frozen so loss.backward() also back-propagates the whole
    trunk (encoder.py:13-17 vs 29-31) -- gradients the optimiser never reads."""
    from oracle import sat_oracle as O
    threads, host = usable_cores()
    torch.set_num_threads(threads)
    B = args.cpu_sample
    enc_p = O.make_resnet152_params(0) if args.network == "resnet152" else O.make_vgg19_params(0)
    fwd = O.resnet152_forward if args.network == "resnet152" else O.vgg19_forward
    D = 2048 if args.network == "resnet152" else 512
    dec_p = O.make_decoder_params(args.vocab, D, 512, True, 0)
    x = torch.randn(B, 3, 224, 224)
    caps = O.make_captions(B, args.seq, args.vocab, 0)

    def run(dead_backward, budget_s, max_iters):
        nonlocal dec_p
        iters, t_total = 0, 0.0
        p_enc = {k: (v.clone().requires_grad_(True) if dead_backward and v.is_floating_point() and "running" not in k
                     else v) for k, v in enc_p.items()}   # conv / BN affine parameters (nn.Parameters)
        while iters < 1 or (t_total < budget_s and iters < max_iters):
            t0 = time.perf_counter()
            if dead_backward:   # train() without no_grad: the trunk's graph is kept and back-propagated
                feats = fwd(p_enc, x)
            else:
                with torch.no_grad():
                    feats = fwd(p_enc, x)
            _, _, dec_p, _, _ = O.train_step(dec_p, feats, caps, tf=not args.no_tf, ado=True, attention=True,
                                             lr=1e-4, training=True, adam_state={})
            t_total += time.perf_counter() - t0
            iters += 1
        return iters, t_total

    run(False, 0.0, 1)   # warm-up (allocator, thread pool)
    it_f, t_f = run(False, 10.0, 20)
    it_d, t_d = run(True, 8.0, 10)
    wl = f"224x224, {args.network} fp32 trunk + decoder train step, V={args.vocab}, T={args.seq}"
    return {"value": round(B * it_f / t_f, 3), "unit": "images/s", "cores": threads, "host_cores": host,
            "batch": B, "kind": "port",
            "sample": f"{it_f} steps x {B} images ({wl}) through oracle/sat_oracle.py on {threads} of the host's "
                      f"{host} cores (the process's CPU affinity / cgroup quota); frozen trunk",
            "reference_as_run": {"value": round(B * it_d / t_d, 3), "unit": "images/s", "steps": it_d,
                                 "note": "the same step with the reference's dead ResNet152 backward (trunk "
                                         "parameters not frozen, encoder.py:13-17)"}}


def decoder_step_roofline(dec, enc, imgs, caps, instep=None, overlapped=None, intervals=None, reps=20):
    """The per-time-step decoder kernels (the fused attention + LSTM step of SURVEY 8(d) and the per-step
    GEMMs) against 8 TB/s: algorithmic bytes per launch / time.  Per group, up to four durations [us]:
    ``us`` (the frac figures) the launch interval -- first start of the launch to the first start of the next
    per-step launch -- from in-kernel timestamps in stamped copies of the decoder graphs replayed on their own
    after the timed region (DecoderStamps, ``intervals``): what a rocprofv3 kernel trace reports per dispatch;
    ``us_span`` the kernels' own first-start / last-end span there (``instep``); ``us_overlapped`` the span
    inside the overlapped schedule; ``us_b2b`` each group of the middle step re-issued ``reps`` times back to
    back between HIP events (sat_decoder_step_bench)."""
    from sat_amd.diagnostics import FUSED, decoder_step_kernels
    with torch.no_grad():
        feats = enc(imgs)
    times_b2b, by = decoder_step_kernels(dec, feats, caps, reps=reps)

    def avg(d):
        return {g: sum(v) / len(v) for g, v in (d or {}).items() if v}
    t_span, t_ov, t_itv = avg(instep), avg(overlapped), avg(intervals)
    primary = t_itv or t_span or times_b2b
    times = {g: primary[g] for g in times_b2b if g in primary and times_b2b[g] > 0}

    def frac(b, us):
        return b / (us * 1e-6) / 1e9 / HBM_PEAK_GBS
    groups = {}
    for g, us in times.items():
        if us <= 0 or by[g] <= 0:
            continue
        groups[g] = {"us": round(us, 2), "mb": round(by[g] / 1e6, 2), "gbs": round(by[g] / (us * 1e-6) / 1e9, 1),
                     "frac": round(frac(by[g], us), 4), "us_b2b": round(times_b2b[g], 2)}
        for key, t in (("us_span", t_span), ("us_overlapped", t_ov)):
            if g in t:
                groups[g][key] = round(t[g], 2)

    def summary(keys):
        keys = [g for g in keys if g in groups]
        by_ = sum(by[g] for g in keys)
        out = {"kernels": keys, "launches_per_step": len(keys)}
        for key, t in (("", times), ("_span", t_span), ("_overlapped", t_ov), ("_b2b", times_b2b)):
            if keys and all(g in t for g in keys):
                us = sum(t[g] for g in keys)
                out[f"us_per_step{key}"] = round(us, 2)
                out[f"frac{key}"] = round(frac(by_, us), 4)
        out["achieved"] = round(by_ / (out["us_per_step"] * 1e-6) / 1e9, 1) if "us_per_step" in out else None
        return out
    src = ("us (frac): launch interval -- first start to the next per-step launch's first start -- from in-kernel "
           "timestamps in stamped copies of the decoder graphs replayed on their own (the per-dispatch duration of "
           "a rocprofv3 kernel trace); us_span: the kernels' own first-start / last-end span there; us_overlapped: "
           "the span inside the overlapped schedule; " if t_itv else "us: ") + \
        f"us_b2b: each group of step (T-1)/2 re-issued {reps}x back to back between HIP events"
    return {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "timing": src, "groups": groups,
            "fused_attention_lstm": summary(FUSED),
            "all_step_kernels": summary(list(groups))}


def fp32_step(args, enc, dec, imgs, caps, pad_id, skip_ids, world):
    """The same train step at the reference's precision (fp32 encoder and decoder: the exact-parity
    path), eager, on this rank's batch; reported beside the bf16 line."""
    import sat_amd
    enc32 = sat_amd.Encoder(args.network, dtype=torch.float32).to(imgs.device).eval()
    enc32.load_state_dict(enc.state_dict())
    opt = sat_amd.Adam(dec.parameters(), lr=1e-4)

    def step():
        with torch.no_grad():
            feats = enc32(imgs)
        opt.zero_grad()
        preds, alphas = dec(feats, caps)
        loss, _ = sat_amd.caption_loss(preds, alphas, caps, pad_id=pad_id, skip_ids=skip_ids)
        loss.backward()
        opt.step()
        return loss

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.fp32_steps):
        loss = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"value": round(imgs.shape[0] * args.fp32_steps / el, 2), "unit": "images/s", "dtype": "fp32",
            "steps": args.fp32_steps, "ms_per_step": round(1000 * el / args.fp32_steps, 2),
            "per_gpu_batch": imgs.shape[0], "loss": round(loss.item(), 4),
            "note": "exact-parity path (fp32 MFMA), eager, rank 0 only; not the headline value"}


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def rank_launch_command(argv, nproc, port):
    """The command that runs this benchmark as `nproc` ranks on one node (one process per GPU over RCCL, or
    several per GPU with --dist-backend gloo): torch.distributed.run with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def launch_ranks(args, argv):
    """--gpus N > 1 outside a torch.distributed.run rank: start the N ranks as a child process and return its exit
    status.  This process never touches the GPU (no HIP call before or after), so the ranks own the devices."""
    import subprocess
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(rank_launch_command(argv, args.gpus, free_port()), env=env).returncode


def dist_info(args, world):
    """the process group the step all-reduces over (N > 1) and the collective library's version"""
    if not dist.is_initialized():
        return {"backend": None, "world_size": 1}
    info = {"backend": dist.get_backend(), "world_size": dist.get_world_size()}
    if info["backend"] == "nccl":   # "nccl" is RCCL on ROCm
        try:
            info["rccl_version"] = ".".join(str(v) for v in torch.cuda.nccl.version())
        except Exception as e:   # noqa: BLE001 -- informational field
            info["rccl_version"] = f"unavailable ({type(e).__name__})"
    return info


# Graph captures run in thread-local capture mode: at N > 1 the RCCL process group's watchdog thread keeps querying
# the events of the warm-up's all-reduces, and under the default (global) mode such a query from another thread
# while this thread captures aborts the process (hipErrorStreamCaptureUnsupported; tests/test_gpu_dp.py's RCCL case)
CAPTURE_MODE = "thread_local"


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched")
    dp = world > 1 or args.dp_rehearse   # the data-parallel path (process group, bucket all-reduces)
    if args.dp_rehearse and world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; --dist-backend gloo rehearses the N > 1 path with several ranks on one GPU
    # (device = LOCAL_RANK modulo the visible GPUs; device_count() does not initialise the GPU)
    local = local % max(1, torch.cuda.device_count())
    if dp:
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    import sat_amd
    from sat_amd.data import synthetic_captions, synthetic_images
    from sat_amd.distributed import GradAllReduce, allreduce_bucket_async, allreduce_grads

    # per-call kernel selection for the A/B flags (None = the library's defaults)
    policy = None
    extra = dict(skinny=1 if args.no_skinny else 0, conv3x3_ws=1 if args.no_ws3x3 else 0,
                 gemm_stages=args.gemm_stages, conv_slices=args.conv_slices)
    for kv in (x for x in args.policy.replace("+", ",").split(",") if x):   # "+" also separates (tools/session.sh)
        k, v = kv.split("=")
        extra[k] = [int(t) for t in v.split(".")] if "." in v else int(v)   # decoder_splits=2.0.0.0
    if any(extra.values()):
        policy = sat_amd.Policy(**extra)
    torch.manual_seed(42 + rank)   # train.py:452 seed; per-rank data stream
    D = 2048 if args.network == "resnet152" else 512
    enc = sat_amd.Encoder(args.network, dtype=torch.bfloat16).to(dev).eval()
    if args.fuse_every is None:
        args.fuse_every = 0   # profiles/r2_s62: none fused 6.79 ms, every 3rd 7.15, every block 7.48
    if args.split_target is None:   # ResNet152 at B = 128: 96 (6.50 vs 6.53 ms; 6.76 vs 6.82 on a slower box), but
        # 64 at B <= 64 (96 there: 4.21-4.23 vs 4.01-4.04 ms), profiles/r3_s46, r3_s47
        args.split_target = 128 if args.network == "vgg19" else (96 if args.batch > 64 else 64)
    enc.fuse_layer2 = args.fuse_layer2
    enc.c2_frag_sizes = tuple(int(v) for v in args.c2_frag_sizes.replace("/", ",").split(",") if v)
    enc.fuse_blocks = (False if args.no_fuse_blocks or args.fuse_every == 0 else
                       (True if args.fuse_every == 1 else args.fuse_every))
    enc.policy = policy
    torch.manual_seed(42)          # identical decoder init on every rank
    dec = sat_amd.Decoder(args.vocab, D, tf=not args.no_tf, ado=not args.bert, bert=args.bert,
                          attention=True).to(dev).train()
    dec.policy = policy
    dec.transposed_weights = not args.no_transposed
    dec.record_tokens = False      # the fed-token record is a diagnostic output, not part of the step
    if not args.no_graph and not args.no_overlap:
        # the decoder shares the chip with the next batch's encoder: fewer split-K workgroups
        dec.split_target = args.split_target
    pad_id, skip_ids = sat_amd.special_ids(args.bert)
    opt = sat_amd.Adam(dec.parameters(), lr=1e-4)
    g = torch.Generator().manual_seed(1000 + rank)
    B = args.batch
    imgs = synthetic_images(B, generator=g, device=dev)
    caps = synthetic_captions(B, args.seq, args.vocab, generator=g, bert=args.bert, device=dev)
    torch.cuda.synchronize()

    def fwd_bwd():
        with torch.no_grad():
            feats = enc(imgs)
        preds, alphas = dec(feats, caps)
        loss, metrics = sat_amd.caption_loss(preds, alphas, caps, pad_id=pad_id, skip_ids=skip_ids)
        loss.backward()
        return loss

    # eager DP: bucket all-reduces launched from inside the decoder's backward (phase hooks)
    grad_ar = GradAllReduce(dec) if dp else None
    # eager warm-up (builds the encoder plan, caches, allocator pools)
    for _ in range(args.warmup):
        opt.zero_grad()
        loss = fwd_bwd()
        if dp:
            grad_ar.wait()
        opt.step()
    torch.cuda.synchronize()
    if grad_ar is not None and not args.no_graph:
        dec._grad_hooks.remove(grad_ar._on_phase)   # graph mode issues the bucket all-reduces itself

    use_graph = not args.no_graph
    overlap = use_graph and not args.no_overlap
    nbuf = args.feature_buffers if overlap else 1
    # backward phase 1 (output head) and phase 2 (BPTT) as two graphs, the head bucket's all-reduce (N > 1)
    # issued between them; --bwd serial: one graph
    split_bwd = dp or args.bwd == "split"
    launches = conv_launches(args.network, B, fused=enc.fuse_blocks, fused2=enc.fuse_layer2)

    def capture(stamped):
        """hipGraphs of the step over ``nbuf`` feature buffers: per buffer the encoder trunk, the decoder's forward +
        loss + backward phase 1 (output head) and, with split_bwd, phase 2 (BPTT + the remaining weight gradients).
        Adam and the RCCL all-reduce run eagerly between replays (Adam's bias corrections are step-dependent host
        scalars).  With overlap (default) the frozen encoder of batch i+1 runs on its own stream while the decoder
        of batch i, its all-reduce and Adam run on the main stream (the encoder reads no decoder parameter).
        stamped: every conv launch and every per-step decoder launch writes in-kernel timestamps (the diagnostic
        copies captured after the timed region; the timed graphs carry no stamp pointers at all)."""
        G = dict(enc=[], dec=[], rec=[], feats=[], loss=[], stamps_enc=[], stamps_dec=[])
        one = torch.ones((), device=dev)
        for k in range(nbuf):
            if stamped:
                G["stamps_enc"].append(LaunchStamps(len(launches), dev, base=policy))
                enc.launch_policy = G["stamps_enc"][-1].next_policy
            g = torch.cuda.CUDAGraph()   # one private memory pool per graph: no intermediate aliases another's
            with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
                with torch.no_grad():
                    G["feats"].append(enc(imgs))
            enc.launch_policy = None
            G["enc"].append(g)
        dec.defer_recurrent_backward(split_bwd)
        for k in range(nbuf):
            if stamped:
                G["stamps_dec"].append(DecoderStamps(args.seq, dev, base=policy))
                dec.policy = G["stamps_dec"][-1].policy
            opt.zero_grad(set_to_none=True)   # each capture overwrites the gradients (beta = 0)
            gd, gr = torch.cuda.CUDAGraph(), None
            with torch.cuda.graph(gd, capture_error_mode=CAPTURE_MODE):
                preds, alphas = dec(G["feats"][k], caps)
                loss_k, _ = sat_amd.caption_loss(preds, alphas, caps, pad_id=pad_id, skip_ids=skip_ids)
                loss_k.backward(one)   # d loss / d loss = 1 from a constant made before capture (no fill node)
            if split_bwd:
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, capture_error_mode=CAPTURE_MODE):
                    dec.finish_backward()
            G["dec"].append(gd)
            G["rec"].append(gr)
            G["loss"].append(loss_k)
            dec.policy = policy
        dec.defer_recurrent_backward(False)
        torch.cuda.synchronize()
        return G

    G = capture(False) if use_graph else None
    enc_events = []
    if overlap and args.stream_priority != "equal":
        lo, hi = torch.cuda.Stream.priority_range()
        dec_hi = args.stream_priority == "decoder-high"
        s_main = torch.cuda.Stream(priority=hi if dec_hi else lo)
        s_enc = torch.cuda.Stream(priority=lo if dec_hi else hi)
        s_main.wait_stream(torch.cuda.current_stream())
        torch.cuda.set_stream(s_main)
    else:
        s_main = torch.cuda.current_stream()
        s_enc = torch.cuda.Stream() if overlap else s_main
    ev_enc = [torch.cuda.Event() for _ in range(max(nbuf, 2))]
    ev_dec = [torch.cuda.Event() for _ in range(max(nbuf, 2))]
    dec_events = []   # (start, end) of each batch's decoder graphs on s_main (after its wait for the features)

    def replay_encoder(G, k, wait_dec):
        """Batch k's encoder on s_enc.  wait_dec: feature buffer k was last read by the decoder nbuf batches ago."""
        with torch.cuda.stream(s_enc):
            if wait_dec:
                s_enc.wait_event(ev_dec[k])
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record(s_enc)
            G["enc"][k].replay()
            en.record(s_enc)
            ev_enc[k].record(s_enc)
        enc_events.append((st, en))

    def run(n, G):
        """n full train steps (encoder fwd, decoder fwd + loss + bwd, all-reduce, Adam)."""
        loss = None
        if G is not None:
            replay_encoder(G, 0, False)
        for i in range(n):
            if G is not None:
                k = i % nbuf
                s_main.wait_event(ev_enc[k])
                d_st, d_en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                d_st.record(s_main)
                G["dec"][k].replay()
                # DP: the output-head bucket is final after phase 1 -> its all-reduce runs on RCCL's
                # stream beside the BPTT graph; the rest follows phase 2
                w1 = allreduce_bucket_async(dec, 1) if dp else None
                if G["rec"][k] is not None:
                    G["rec"][k].replay()
                w2 = allreduce_bucket_async(dec, 2) if dp else None
                d_en.record(s_main)
                dec_events.append((d_st, d_en))
                ev_dec[k].record(s_main)
                loss = G["loss"][k]
                if i + 1 < n:
                    if overlap:   # buffer (i + 1) % nbuf was last read by batch i + 1 - nbuf's decoder
                        replay_encoder(G, (i + 1) % nbuf, i >= nbuf - 1)
                    else:
                        replay_encoder(G, 0, False)
                if dp:
                    w1.wait()
                    w2.wait()
            else:
                opt.zero_grad()
                loss = fwd_bwd()
                if dp:
                    grad_ar.wait()
            opt.step()
        return loss

    run(2, G)   # replay warm-up
    enc_events.clear()
    dec_events.clear()
    torch.cuda.synchronize()
    if dp:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss = run(args.steps, G)
    torch.cuda.synchronize()
    if dp:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dp:
        t = torch.tensor([elapsed], device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    loss_v = loss.item()
    enc_ms = sum(s.elapsed_time(e) for s, e in enc_events) if use_graph else None
    dec_ms = sum(s.elapsed_time(e) for s, e in dec_events) if use_graph and dec_events else None
    diag_phase = None
    stamps_enc, stamps_dec = [], []
    if use_graph and not args.no_diagnostics and not args.no_step_stamps:
        # diagnostic phase (every rank: the all-reduces are collective): stamped copies of the graphs, captured
        # now (the timed graphs are released first), run in the same overlapped schedule with the timestamps on
        loss = None
        G = None
        torch.cuda.synchronize()
        G = capture(True)
        stamps_enc, stamps_dec = G["stamps_enc"], G["stamps_dec"]
        run(2, G)
        for st in stamps_enc + stamps_dec:
            st.enable(True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        n_diag = max(4, min(20, args.steps))
        run(n_diag, G)
        torch.cuda.synchronize()
        diag_phase = {"steps": n_diag, "ms_per_step": round(1000 * (time.perf_counter() - t1) / n_diag, 3)}
        for st in stamps_enc + stamps_dec:
            st.enable(False)
    diag = rank == 0 and not args.no_diagnostics

    def collect(intervals=False):
        conv = instep_conv_durations(stamps_enc, launches, intervals=intervals) if stamps_enc else None
        decd = None
        if stamps_dec:
            decd = {}
            for sd in stamps_dec:
                for g, v in (sd.group_intervals_us() if intervals else sd.group_spans_us()).items():
                    decd.setdefault(g, []).extend(v)
        return conv, decd

    def chains():   # the per-step chain figures, averaged over the graph sets
        cs = [sd.chain_us() for sd in stamps_dec]
        keys = {k for c in cs for k in c}
        return {k: round(sum(c[k] for c in cs if k in c) / sum(1 for c in cs if k in c), 2) for k in sorted(keys)}
    overlap_conv, overlap_dec = collect() if diag_phase else (None, None)
    chain_overlapped = chains() if diag_phase and stamps_dec else None
    chain_alone = None
    alone_conv = alone_dec = alone_intervals = alone_dec_intervals = None
    if diag and diag_phase:
        # graph-alone phase: each encoder graph, then each decoder graph pair, replayed on its own (nothing
        # beside it) with the timestamps on -- the kernels' durations as a rocprofv3 kernel trace of this
        # command sees them (the trace all but serialises the two streams); the overlapped figures above
        # stay as the secondary in-step keys
        for st in stamps_enc + stamps_dec:
            st.enable(True)
        torch.cuda.synchronize()
        for k in range(nbuf):
            for _ in range(3):
                G["enc"][k].replay()
                torch.cuda.synchronize()
            for _ in range(3):
                G["dec"][k].replay()
                if G["rec"][k] is not None:
                    G["rec"][k].replay()
                torch.cuda.synchronize()
        alone_conv, alone_dec = collect()
        alone_intervals, alone_dec_intervals = collect(intervals=True)
        chain_alone = chains() if stamps_dec else None
        for st in stamps_enc + stamps_dec:
            st.enable(False)
    roof, trunk = trunk_roofline(enc, imgs, launches, instep=alone_conv or overlap_conv,
                                 overlapped=overlap_conv, intervals=alone_intervals) if diag else (None, None)
    step_kernels = decoder_step_roofline(dec, enc, imgs, caps, instep=alone_dec or overlap_dec,
                                         overlapped=overlap_dec, intervals=alone_dec_intervals) if diag else None
    if step_kernels is not None and (chain_alone or chain_overlapped):
        step_kernels["step_chain"] = dict(alone=chain_alone, overlapped=chain_overlapped,
                                          note="per time step: first-kernel start to the next step's first-kernel "
                                               "start (interval) beside the sum of the step's kernel spans")
    fp32_leg = fp32_step(args, enc, dec, imgs, caps, pad_id, skip_ids, world) if world == 1 and args.fp32_steps > 0 \
        else None
    if roof is not None:
        roof["traffic"], roof["traffic_source"] = pmc_traffic(args.network, roof["cls"])
    if rank == 0:
        # the whole step's algorithmic FLOPs (encoder fwd + decoder fwd/bwd with W.a
        # hoisted) per image x images / step time, against the dense bf16 MFMA peak
        from sat_amd.diagnostics import decoder_flops
        D = 2048 if args.network == "resnet152" else 512
        Lf = 49 if args.network == "resnet152" else 196
        E = 768 if args.bert else 512
        enc_f = sum(l["flops"] for l in launches) / B
        dec_f = decoder_flops(Lf, D, E, args.vocab, args.seq, ado=not args.bert, attention=True)
        step_tf = (enc_f + dec_f) * B * world * args.steps / elapsed / 1e12
        if roof is not None:
            roof["step"] = {"encoder_gflop_per_img": round(enc_f / 1e9, 3),
                            "decoder_gflop_per_img": round(dec_f / 1e9, 3), "achieved": round(step_tf, 1),
                            "peak": BF16_DENSE_PEAK_TFLOPS, "unit": "TFLOP/s",
                            "frac": round(step_tf / BF16_DENSE_PEAK_TFLOPS, 4)}
            roof["decoder_step_kernels"] = step_kernels
        out = {
            "metric": "train images/sec on COCO batch=128 at 1/2/4/8 MI355X",
            "value": round(B * world * args.steps / elapsed, 2),
            "unit": "images/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "dist": dist_info(args, world),
            "ms_per_step": round(1000 * elapsed / args.steps, 3),
            "timing": ("host wall clock (perf_counter) around exactly `steps` pipelined train steps, bracketed by a "
                       "barrier + device synchronize on both sides, max over ranks; a step's encoder runs beside "
                       "the previous batch's decoder, so per-step device times are not separable -- the mean over "
                       "the window, not a per-step event median"),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            # this line measures one point of the curve: per-GPU work is fixed (weak scaling), and the 1 -> 8 curve
            # exists only where the driver's SCALE runs (N = 1, 2, 4, 8 on one node) measured it
            "scaling_curve": ("unmeasured: N = 1 only (the 2 / 4 / 8-GPU points come from the driver's SCALE runs)"
                              if world == 1 else f"one point, N = {world}"),
            "dtype": "bf16", "data": "synthetic (224x224 N(0,1) images, random-token captions, random-init weights)",
            "config": {"workload": f"{'Flickr8k' if args.bert else 'COCO'}-shaped {args.network} encoder (bf16 fwd) + attention/{'greedy' if args.no_tf else 'tf'}/{'bert' if args.bert else 'ado'} decoder train "
                                   f"step, V={args.vocab}, T={args.seq}",
                       "global_batch": B * world, "per_gpu_batch": B, "seq_len": args.seq,
                       "parallelism": f"dp{world}", "hip_graph": use_graph,
                       "encoder_decoder_overlap": overlap},
            "roofline": roof,
            "diagnostic_phase": dict(diag_phase, note="after the timed region: the same overlapped graphs with the "
                                     "kernels' in-kernel timestamps on (roofline in-step figures)") if diag_phase else None,
            "decoder_graphs_ms_per_step": round(dec_ms / args.steps, 3) if dec_ms else None,
            "encoder_trunk": dict(trunk or {}, graph_ms_per_step=(round(enc_ms / args.steps, 3) if enc_ms else None)),
            "loss": round(loss_v, 4),
        }
        if fp32_leg is not None:
            out["fp32"] = fp32_leg
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    if dp:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
