"""Data-parallel path on CPU with gloo, world_size 2 (the MI355X run uses RCCL).

(1) The bucketed gradient all-reduce helpers average the decoder's flat gradient buckets.
(2) The DP step is equivalent to the full-batch step: the mean of per-rank gradients of the
    reference loss on B/2-image shards equals the gradient on the full batch (both loss terms
    are means over equal-size local sets) -- checked with the CPU oracle.
"""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import sat_oracle as O


class FakeDecoder:
    def __init__(self, rank):
        self._grad_hooks = []
        self.head = torch.full((10,), float(rank + 1))
        self.rest = torch.arange(6, dtype=torch.float32) * (rank + 1)

    def grad_bucket(self, phase):
        return self.head if phase == 1 else self.rest


def _worker(rank, world, init_file, results):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    import sat_amd.distributed as D
    torch.set_num_threads(1)
    # (1a) synchronous helper
    fake = FakeDecoder(rank)
    D.allreduce_grads(fake)
    ok1 = torch.allclose(fake.head, torch.full((10,), 1.5)) and torch.allclose(fake.rest, torch.arange(6.) * 1.5)
    # (1b) hook-driven async buckets
    fake2 = FakeDecoder(rank)
    r = D.GradAllReduce(fake2)
    for phase in (1, 2):
        for hook in fake2._grad_hooks:
            hook(phase, fake2)
    r.wait()
    ok2 = torch.allclose(fake2.head, torch.full((10,), 1.5))
    # (2) sharded gradients == full-batch gradients
    V, D_, E, B, T = 40, 16, 512, 4, 7
    p = O.make_decoder_params(V, D_, E, True, 3)
    feats = torch.from_numpy(__import__("numpy").random.default_rng(5).standard_normal((B, 6, D_)).astype("float32"))
    caps = O.make_captions(B, T, V, 9)
    shard = slice(rank * B // world, (rank + 1) * B // world)
    _, g_local, _, _, _ = O.train_step(p, feats[shard], caps[shard], tf=True, ado=True, attention=True,
                                       training=False)
    _, g_full, _, _, _ = O.train_step(p, feats, caps, tf=True, ado=True, attention=True, training=False)
    ok3 = True
    for k in sorted(g_full):
        g = g_local[k].clone()
        dist.all_reduce(g)
        g /= world
        scale = g_full[k].abs().max().item()
        if scale > 1e-7 and (g - g_full[k]).abs().max().item() > 1e-4 * scale:
            ok3 = False
    results[rank] = (ok1, ok2, ok3)
    dist.destroy_process_group()


def test_gloo_world_size_2():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        init_file = os.path.join(d, "init")
        mgr = mp.Manager()
        results = mgr.dict()
        mp.spawn(_worker, args=(world, init_file, results), nprocs=world, join=True)
        assert dict(results) == {0: (True, True, True), 1: (True, True, True)}
