"""Data parallelism: one process per GPU, RCCL gradient all-reduce over xGMI.

The reference is single-device (no torch.distributed).  Each rank
runs the same train step on its own B/N images; the decoder gradients are
averaged across ranks between backward and Adam, which reproduces the
full-batch step because both loss terms are means over equal-size local sets
(SURVEY 8e).

Two buckets, launched asynchronously as soon as each is final:
  * bucket 1 = the output head (f_out/f_h/f_z or deep_output), ready right after
    backward phase 1, so its all-reduce overlaps the whole recurrent BPTT;
  * bucket 2 = everything else, ready when BPTT finishes.
Both are contiguous slices of the decoder's flat gradient buffer: no packing.
Eager training (train.py) uses GradAllReduce, whose hooks fire from inside the
decoder's backward; the hipGraph path (bench.py) captures phase 1 and phase 2 as two
graphs (Decoder.defer_recurrent_backward) and calls allreduce_bucket_async between
their replays.
"""
import torch
import torch.distributed as dist


class GradAllReduce:
    def __init__(self, decoder, group=None):
        self.decoder = decoder
        self.group = group
        self.world = dist.get_world_size(group)
        self.works = []
        self.buckets = []
        self.use_avg = dist.get_backend(group) == "nccl"   # RCCL has ncclAvg; gloo does not
        decoder._grad_hooks.append(self._on_phase)

    def _on_phase(self, phase, dec):
        bucket = dec.grad_bucket(phase)
        op = dist.ReduceOp.AVG if self.use_avg else dist.ReduceOp.SUM
        self.works.append(dist.all_reduce(bucket, op=op, group=self.group, async_op=True))
        self.buckets.append(bucket)

    def wait(self):
        for w in self.works:
            w.wait()
        if not self.use_avg:
            for b in self.buckets:
                b.div_(self.world)
        self.works, self.buckets = [], []


def shard_batch(tensor, rank, world):
    """Rank r's contiguous 1/N of a global batch (global batch divisible by N)."""
    n = tensor.shape[0]
    if n % world:
        raise ValueError(f"global batch {n} not divisible by world size {world}")
    per = n // world
    return tensor[rank * per:(rank + 1) * per]


def allreduce_bucket_async(decoder, phase, group=None):
    """Start the mean all-reduce of one gradient bucket; returns a handle whose wait() makes the
    current stream wait for it (RCCL runs on its own stream, ordered after the work already queued
    on the current stream -- e.g. the replayed graph that produced the bucket)."""
    bucket = decoder.grad_bucket(phase)
    avg = dist.get_backend(group) == "nccl"
    work = dist.all_reduce(bucket, op=dist.ReduceOp.AVG if avg else dist.ReduceOp.SUM, group=group, async_op=True)
    world = dist.get_world_size(group)

    class _Handle:
        def wait(self):
            work.wait()
            if not avg:
                bucket.div_(world)
    return _Handle()


def allreduce_grads(decoder, group=None):
    """Synchronous mean all-reduce of the decoder's two gradient buckets (used after a hipGraph
    replay of fwd+bwd, where the in-backward hooks of GradAllReduce cannot run)."""
    world = dist.get_world_size(group)
    avg = dist.get_backend(group) == "nccl"
    for phase in (1, 2):
        bucket = decoder.grad_bucket(phase)
        dist.all_reduce(bucket, op=dist.ReduceOp.AVG if avg else dist.ReduceOp.SUM, group=group)
        if not avg:
            bucket.div_(world)
