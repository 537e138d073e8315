"""One rank of the data-parallel GPU test (tests/test_gpu_dp.py launches two of these, gloo, both on
cuda:0, or one over RCCL: SAT_DP_BACKEND=nccl).  Not a test module: run as
``python tests/dp_rank_worker.py RANK WORLD INIT_FILE OUT [CASE]`` (CASE: a DP_CASES key).

Each rank takes its contiguous half of a global fp32 batch and runs the train step (train.py:128-164)
through the HIP decoder twice:
  eager  -- backward with GradAllReduce's phase hooks (bucket 1 all-reduced from inside backward);
  graph  -- bench.py's schedule: forward + loss + backward phase 1 captured as one hipGraph, phase 2
            (BPTT) as a second, allreduce_bucket_async between / after the replays;
each followed by the fused Adam step.  It also runs one train-mode forward with library-drawn dropout
masks on the SAME inputs on every rank (the per-rank mask streams must differ, decoder.py:121-125
draws a fresh Bernoulli mask per sample).  Results go to OUT (torch.save) for the parent to compare
with a single-process full-batch run.
"""
import os
import sys

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

DP_CASES = {
    # toy fp32 (the exact-parity path) and cfg3's per-rank shape: COCO ResNet152 features (L 49, D 2048), V 10000,
    # T 27, bf16, 64 images per rank with bench.py's split target for B <= 64 (BASELINE cfg3: B = 512 over 8 GPUs)
    "toy_fp32": dict(V=500, D=256, L=16, E=512, T=10, B=8, seed=41, lr=1e-4, bf16=False, split_target=0),
    "cfg3_bf16": dict(V=10000, D=2048, L=49, E=512, T=27, B=128, seed=43, lr=1e-4, bf16=True, split_target=64),
}
DP_CASE = DP_CASES["toy_fp32"]


def case_inputs(c=DP_CASE):
    import numpy as np
    from oracle import sat_oracle as O
    p = O.make_decoder_params(c["V"], c["D"], c["E"], True, c["seed"])
    rng = np.random.default_rng(c["seed"] + 1)
    feats = torch.from_numpy(np.maximum(rng.standard_normal((c["B"], c["L"], c["D"])), 0).astype(np.float32))
    if c["bf16"]:
        feats = feats.bfloat16()
    caps = O.make_captions(c["B"], c["T"], c["V"], c["seed"] + 2)
    masks = O.make_dropout_masks(c["B"], c["T"] - 1, c["E"], c["seed"] + 3)   # [T-1, B, E]
    return p, feats, caps, masks.permute(1, 0, 2).contiguous().to(torch.uint8)   # [B, T-1, E]


def make_decoder(sat_amd, p, dev, c=DP_CASE):
    dec = sat_amd.Decoder(c["V"], c["D"], tf=True, ado=True, attention=True)
    dec.load_state_dict(p, strict=True)
    dec.split_target = c["split_target"]
    return dec.to(dev).train()


def snapshot(dec):
    params = dict(dec.named_parameters())
    return {n: params[n].grad.detach().cpu().clone() for n in dec.active_param_names()}


def weights(dec):
    params = dict(dec.named_parameters())
    return {n: params[n].detach().cpu().clone() for n in dec.active_param_names()}


def main():
    rank, world, init_file, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    c = DP_CASES[sys.argv[5] if len(sys.argv) > 5 else "toy_fp32"]
    backend = os.environ.get("SAT_DP_BACKEND", "gloo")   # "nccl" is RCCL on ROCm (one rank per GPU)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", init_method=f"file://{init_file}", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    import sat_amd
    from sat_amd.distributed import GradAllReduce, allreduce_bucket_async, shard_batch
    p, feats, caps, mask = case_inputs(c)
    f_loc = shard_batch(feats, rank, world).contiguous().to(dev)
    c_loc = shard_batch(caps, rank, world).contiguous().to(dev)
    m_loc = shard_batch(mask, rank, world).contiguous().to(dev)   # on the device: no copy inside a capture
    res = {"backend": dist.get_backend()}
    if backend == "nccl":
        res["rccl_version"] = ".".join(str(v) for v in torch.cuda.nccl.version())

    # -- eager: hook-driven bucket all-reduce
    dec = make_decoder(sat_amd, p, dev, c)
    dec.dropout_mask = m_loc
    opt = sat_amd.Adam(dec.parameters(), lr=c["lr"])
    ar = GradAllReduce(dec)
    opt.zero_grad()
    preds, alphas = dec(f_loc, c_loc)
    loss, _ = sat_amd.caption_loss(preds, alphas, c_loc)
    loss.backward()
    ar.wait()
    torch.cuda.synchronize()
    res["eager_grads"] = snapshot(dec)
    opt.step()
    torch.cuda.synchronize()
    res["eager_weights"] = weights(dec)

    # -- graph: two captured decoder graphs (phase 1, phase 2), async bucket all-reduce between
    dec = make_decoder(sat_amd, p, dev, c)
    dec.dropout_mask = m_loc
    opt = sat_amd.Adam(dec.parameters(), lr=c["lr"])
    opt.zero_grad()   # warm-up eager step: builds the flat buffers and the allocator pools
    preds, alphas = dec(f_loc, c_loc)
    sat_amd.caption_loss(preds, alphas, c_loc)[0].backward()
    torch.cuda.synchronize()
    dec.defer_recurrent_backward(True)
    opt.zero_grad(set_to_none=True)
    g_dec, g_rec = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    # thread-local capture: the RCCL watchdog thread may still query the eager all-reduces' events (bench.py)
    with torch.cuda.graph(g_dec, capture_error_mode="thread_local"):
        preds, alphas = dec(f_loc, c_loc)
        sat_amd.caption_loss(preds, alphas, c_loc)[0].backward()
    with torch.cuda.graph(g_rec, capture_error_mode="thread_local"):
        dec.finish_backward()
    dec.defer_recurrent_backward(False)
    dec._grad_flat.fill_(float("nan"))   # every replay must overwrite the whole gradient
    g_dec.replay()
    w1 = allreduce_bucket_async(dec, 1)
    g_rec.replay()
    w2 = allreduce_bucket_async(dec, 2)
    w1.wait()
    w2.wait()
    torch.cuda.synchronize()
    res["graph_grads"] = snapshot(dec)
    opt.step()
    torch.cuda.synchronize()
    res["graph_weights"] = weights(dec)

    # -- library-drawn dropout masks: identical inputs and weights on every rank
    dec = make_decoder(sat_amd, p, dev, c)
    same_f, same_c = feats[:2].contiguous().to(dev), caps[:2].contiguous().to(dev)
    with torch.no_grad():
        res["train_preds"] = dec(same_f, same_c)[0].cpu()
        dec.eval()
        res["eval_preds"] = dec(same_f, same_c)[0].cpu()
    torch.save(res, out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
