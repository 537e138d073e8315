"""Benchmark: train images/sec of the Show-Attend-and-Tell step on MI355X.

Workload (BASELINE.json metric "train images/sec on COCO batch=128 at 1/2/4/8 MI355X"):
COCO-shaped synthetic batches -- 128 images/GPU of 224x224 (weak scaling), ResNet152
encoder (bf16, forward), decoder with --attention --tf --ado (E=512, D=2048, L=49),
V=10000, T=27 caption slots; random-init weights (no checkpoints offline).
One step = encoder fwd + decoder fwd + fused loss + decoder bwd + RCCL grad
all-reduce (N>1) + Adam, inputs resident in HBM before the timed region.

Run:  python bench.py [--gpus N --steps K --warmup W]
      (N>1 via: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...)
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=128, help="images per GPU")
    ap.add_argument("--network", default="resnet152", choices=["resnet152", "vgg19"])
    ap.add_argument("--vocab", type=int, default=10000)
    ap.add_argument("--seq", type=int, default=27)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=2, help="images in the bounded CPU-baseline sample")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraph replay")
    return ap.parse_args()


def conv_flops(enc, B, H=224, W=224):
    """Algorithmic FLOPs of every conv launch of one encoder forward (real Cin, not the padded one)."""
    flops = []
    h, w = H, W
    for step in enc._plan:   # the plan the timed steps ran (built during warm-up)
        if step[0] == "conv":
            wt, _, s, p = step[1]
            co, kh, kw, ci = wt.shape
            ci = 3 if ci == 8 else ci
            oh, ow = (h + 2 * p - kh) // s + 1, (w + 2 * p - kw) // s + 1
            flops.append(2.0 * B * oh * ow * co * kh * kw * ci)
            h, w = oh, ow
        elif step[0] == "pool":
            k, s, p = step[1], step[2], step[3]
            h, w = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        else:
            _, c1, c2, c3, ds = step
            s = c2[2]
            oh, ow = (h + 2 - 3) // s + 1, (w + 2 - 3) // s + 1
            for (wt, _, st, pd), (hh, ww, oo) in ((c1, (h, w, (h, w))), (c2, (h, w, (oh, ow))),
                                                   (c3, (oh, ow, (oh, ow)))):
                co, kh, kw, ci = wt.shape
                flops.append(2.0 * B * oo[0] * oo[1] * co * kh * kw * ci)
            if ds is not None:
                co, kh, kw, ci = ds[0].shape
                flops.append(2.0 * B * oh * ow * co * ci)
            h, w = oh, ow
    return flops


def pmc_traffic(network):
    """HBM bytes per conv launch from the committed PMC passes (tools/pmc_traffic.py; a PMC run
    cannot share a process with the timed bench), or None when none was collected for this trunk."""
    path = os.path.join(REPO, "profiles", f"pmc_traffic_{network}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        rec = json.load(f)
    return rec.get("hbm_bytes_per_conv_launch"), os.path.relpath(path, REPO)


def cpu_baseline(args):
    """Bounded CPU sample of the same step through the oracle (torch-CPU fp32 port)."""
    from oracle import sat_oracle as O
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    B = args.cpu_sample
    enc_p = O.make_resnet152_params(0) if args.network == "resnet152" else O.make_vgg19_params(0)
    fwd = O.resnet152_forward if args.network == "resnet152" else O.vgg19_forward
    D = 2048 if args.network == "resnet152" else 512
    dec_p = O.make_decoder_params(args.vocab, D, 512, True, 0)
    x = torch.randn(B, 3, 224, 224)
    caps = O.make_captions(B, args.seq, args.vocab, 0)
    iters, t_total = 0, 0.0
    while iters < 2 or (t_total < 10.0 and iters < 5):
        t0 = time.perf_counter()
        with torch.no_grad():
            feats = fwd(enc_p, x)
        _, _, dec_p, _, _ = O.train_step(dec_p, feats, caps, tf=True, ado=True, attention=True, lr=1e-4,
                                         training=True, adam_state={})
        t_total += time.perf_counter() - t0
        iters += 1
    return {"value": round(B * iters / t_total, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{iters} steps x {B} images (224x224, {args.network} fp32 trunk + decoder train step, "
                      f"V={args.vocab}, T={args.seq}) through oracle/sat_oracle.py on host CPU"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    import sat_amd
    from sat_amd.data import synthetic_captions, synthetic_images
    from sat_amd.distributed import allreduce_grads

    torch.manual_seed(42 + rank)   # train.py:452 seed; per-rank data stream
    D = 2048 if args.network == "resnet152" else 512
    enc = sat_amd.Encoder(args.network, dtype=torch.bfloat16).to(dev).eval()
    torch.manual_seed(42)          # identical decoder init on every rank
    dec = sat_amd.Decoder(args.vocab, D, tf=True, ado=True, attention=True).to(dev).train()
    opt = sat_amd.Adam(dec.parameters(), lr=1e-4)
    g = torch.Generator().manual_seed(1000 + rank)
    B = args.batch
    imgs = synthetic_images(B, generator=g, device=dev)
    caps = synthetic_captions(B, args.seq, args.vocab, generator=g, device=dev)
    torch.cuda.synchronize()

    def fwd_bwd():
        with torch.no_grad():
            feats = enc(imgs)
        preds, alphas = dec(feats, caps)
        loss, metrics = sat_amd.caption_loss(preds, alphas, caps)
        loss.backward()
        return loss

    # eager warm-up (builds the encoder plan, caches, allocator pools)
    for _ in range(args.warmup):
        opt.zero_grad()
        loss = fwd_bwd()
        if world > 1:
            allreduce_grads(dec)
        opt.step()
    torch.cuda.synchronize()

    use_graph = not args.no_graph
    if use_graph:
        # Two hipGraphs: the encoder trunk (so its kernels can be bracketed with events) and
        # decoder fwd + loss + BPTT.  Adam and the RCCL all-reduce run eagerly after replay
        # (Adam's bias corrections are step-dependent host scalars).
        opt.zero_grad(set_to_none=True)
        g_enc, g_dec = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_enc):
            with torch.no_grad():
                feats_static = enc(imgs)
        with torch.cuda.graph(g_dec, pool=g_enc.pool()):
            preds, alphas = dec(feats_static, caps)
            loss_static, _ = sat_amd.caption_loss(preds, alphas, caps)
            loss_static.backward()
        torch.cuda.synchronize()

    enc_events = []

    def step():
        if use_graph:
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            g_enc.replay()
            en.record()
            enc_events.append((st, en))
            g_dec.replay()
            loss = loss_static
        else:
            opt.zero_grad()
            loss = fwd_bwd()
        if world > 1:
            allreduce_grads(dec)
        opt.step()
        return loss

    for _ in range(2):   # replay warm-up
        step()
    enc_events.clear()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if not use_graph:
        enc.timing = []   # eager: bracket every conv launch
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    per_img_conv = conv_flops(enc, B)
    if use_graph:
        enc_ms = sum(s.elapsed_time(e) for s, e in enc_events)
        n_launch = len(per_img_conv) * args.steps
        kernel_desc = "encoder trunk hipGraph (155 implicit-GEMM conv launches fast_gemm_kernel<*,0,0,2,8> + pool/layout)"
    else:
        enc_ms = sum(s.elapsed_time(e) for s, e in enc.timing)
        n_launch = len(enc.timing)
        enc.timing = None
        kernel_desc = "fast_gemm_kernel<*,0,0,2,8> (implicit-GEMM conv), per-launch events"
    flops = sum(per_img_conv) * args.steps
    achieved = flops / (enc_ms * 1e-3) / 1e12 if enc_ms > 0 else 0.0
    loss_v = loss.item()
    traffic, t_src = pmc_traffic(args.network)
    if rank == 0:
        out = {
            "metric": "train images/sec on COCO batch=128 at 1/2/4/8 MI355X",
            "value": round(B * world * args.steps / elapsed, 2),
            "unit": "images/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16", "data": "synthetic (224x224 N(0,1) images, random-token captions, random-init weights)",
            "config": {"workload": f"COCO-shaped {args.network} encoder (bf16 fwd) + attention/tf/ado decoder train "
                                   f"step, V={args.vocab}, T={args.seq}",
                       "global_batch": B * world, "per_gpu_batch": B, "seq_len": args.seq,
                       "parallelism": f"dp{world}", "hip_graph": use_graph},
            "roofline": {"bound": "mfma", "kernel": kernel_desc,
                         "achieved": round(achieved, 2), "peak": BF16_DENSE_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / BF16_DENSE_PEAK_TFLOPS, 4),
                         "launches": n_launch, "avg_launch_ms": round(enc_ms / max(1, n_launch), 4),
                         "algorithmic_flops_per_launch": flops / max(1, n_launch),
                         "traffic": traffic, "traffic_unit": "HBM bytes per conv launch", "traffic_source": t_src},
            "loss": round(loss_v, 4),
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
