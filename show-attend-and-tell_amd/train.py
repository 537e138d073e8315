"""Training CLI with the reference's flags (train.py:438-472) on the MI355X path.

    python show-attend-and-tell_amd/train.py --data data/flickr8k --network vgg19 --tf --ado --attention
    python show-attend-and-tell_amd/train.py --synthetic 512 --network resnet152 --tf --ado --attention

Same flags and defaults as the reference (``--perform-test`` is store_true with default True,
so it cannot be disabled, as in train.py:450), plus:
  --synthetic N   N synthetic images (5 captions each is not needed: one caption per row) instead
                  of the Karpathy-JSON dataset;  --vocab for its vocabulary size
  --dtype         bf16 (default, performance) | fp32 (exact parity mode)
  --max-steps     cap batches per epoch (smoke runs)
  --no-overlap    encode each batch just before its decoder step (default: the frozen encoder of
                  batch i+1 runs on a side stream beside batch i's decoder step)
  --encoder-weights  torchvision-layout state_dict of the trunk (weights_only load); without it the
                  trunk is randomly initialised under --seed (no pretrained weights offline).  Either
                  way the trunk actually used is saved as <out>/encoder_<network>.pth and recorded in
                  model_config.json, so generate_caption.py runs the same encoder
  --host-preprocess  resize + normalize on the DataLoader workers (default: workers only decode, the
                  uint8 images travel at native size and sat_images_to_input resamples them on the GPU,
                  bit-identical to PIL's bilinear resize + torchvision's ToTensor / Normalize)
  --workers       decode workers per rank (default 8)
  --bert-embeddings  a local [30522, 768] bert-base-uncased word-embedding table (a tensor, or a
                  state_dict holding embeddings.word_embeddings.weight / embedding.weight)
Multi-GPU: ``python -m torch.distributed.run --nproc-per-node N show-attend-and-tell_amd/train.py ...``
(RCCL data parallel; the batch size is per GPU).  W&B logging is not part of this build; the
reference's scalar names are printed / written as JSON lines instead.
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import sat_amd  # noqa: E402
else:
    import sat_amd  # noqa: E402
from sat_amd import bleu as bleu_mod  # noqa: E402
from sat_amd import distributed as sat_dist  # noqa: E402
from sat_amd.data import synthetic_captions, synthetic_images  # noqa: E402

MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)   # train.py:27-32
STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


class AverageMeter:
    """utils.py:4-19"""

    def __init__(self):
        self.val = self.avg = self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count if self.count else 0


class JsonCaptionDataset(torch.utils.data.Dataset):
    """The reference's on-disk layout (generate_json_data.py:51-63, dataset.py:15-52), loaded
    lazily per item (the reference decodes every image eagerly into RAM, which does not fit COCO)."""

    def __init__(self, data_path, split_type="train", fraction=1.0, bert=False, decode_only=False):
        self.decode_only = decode_only   # uint8 HWC at native size; resize + normalize run on the GPU
        self.paths = json.load(open(os.path.join(data_path, f"{split_type}_img_paths.json")))
        name = f"{split_type}_captions_bert.json" if bert else f"{split_type}_captions.json"
        self.captions = json.load(open(os.path.join(data_path, name)))
        if fraction != 1.0:
            self.paths = self.paths[:int(len(self.paths) * fraction)]
            self.captions = self.captions[:int(len(self.captions) * fraction)]
        by_path = {}
        for p, c in zip(self.paths, self.captions):
            by_path.setdefault(p, []).append(c)
        self.all_captions = [by_path[p] for p in self.paths]

    def __len__(self):
        return len(self.paths)

    def __getitem__(self, i):
        from PIL import Image
        with open(self.paths[i], "rb") as f:   # dataset.py:9-12
            img = Image.open(f).convert("RGB")
        caps = torch.tensor(self.captions[i]), torch.tensor(self.all_captions[i])
        if self.decode_only:
            return (np.asarray(img, dtype=np.uint8),) + caps
        img = img.resize((224, 224), Image.BILINEAR)   # host transform (train.py:27-32), --host-preprocess
        x = (np.asarray(img, dtype=np.float32) / 255.0 - MEAN) / STD
        return (torch.from_numpy(x.transpose(2, 0, 1).copy()),) + caps


class SyntheticDataset(torch.utils.data.Dataset):
    def __init__(self, n, vocab, T, bert, seed):
        g = torch.Generator().manual_seed(seed)
        self.caps = synthetic_captions(n, T, vocab, generator=g, bert=bert)
        self.seed = seed

    def __len__(self):
        return self.caps.shape[0]

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 100003 + i)
        return synthetic_images(1, generator=g)[0], self.caps[i], self.caps[i:i + 1]


def set_seed(seed):
    """train.py:37-43"""
    torch.manual_seed(seed)
    np.random.seed(seed)
    random.seed(seed)


def parse(argv=None):
    p = argparse.ArgumentParser(description="Show, Attend and Tell (MI355X)")
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--epochs", type=int, default=10)
    p.add_argument("--lr", type=float, default=1e-4)
    p.add_argument("--step-size", type=int, default=5)
    p.add_argument("--alpha-c", type=float, default=1)
    p.add_argument("--perform-test", action="store_true", default=True)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--log-interval", type=int, default=100)
    p.add_argument("--data", type=str, default="data/coco")
    p.add_argument("--network", choices=["vgg19", "resnet152", "densenet161"], default="vgg19")
    p.add_argument("--model", type=str)
    p.add_argument("--tf", action="store_true", default=False)
    p.add_argument("--ado", action="store_true", default=False)
    p.add_argument("--fraction", type=float, default=1.0)
    p.add_argument("--bert", action="store_true", default=False)
    p.add_argument("--attention", action="store_true", default=False)
    # MI355X build
    p.add_argument("--synthetic", type=int, default=0)
    p.add_argument("--vocab", type=int, default=10000)
    p.add_argument("--seq", type=int, default=27)
    p.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    p.add_argument("--max-steps", type=int, default=0)
    p.add_argument("--out", type=str, default="model")
    p.add_argument("--no-overlap", action="store_true",
                   help="encode each batch right before its decoder step instead of one batch ahead on a side stream")
    p.add_argument("--encoder-weights", type=str, default=None,
                   help="torchvision-layout encoder state_dict (weights_only); default: random init under --seed")
    p.add_argument("--host-preprocess", action="store_true",
                   help="resize + normalize on the host workers (default: workers only decode; the GPU resamples "
                        "the uint8 images bit-identically to PIL and normalizes into the encoder's input layout)")
    p.add_argument("--workers", type=int, default=8, help="DataLoader decode workers per rank")
    p.add_argument("--bert-embeddings", type=str, default=None,
                   help="local bert-base-uncased word-embedding table [30522, 768] (weights_only)")
    return p.parse_args(argv)


def load_bert_embeddings(path):
    """The frozen BERT word-embedding table the reference takes from BertModel.from_pretrained
    (decoder.py:21-36), from a local file: a tensor or a state_dict holding it."""
    obj = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(obj, dict):
        for k in ("embeddings.word_embeddings.weight", "bert.embeddings.word_embeddings.weight",
                  "word_embeddings.weight", "embedding.weight", "weight"):
            if k in obj:
                obj = obj[k]
                break
        else:
            raise ValueError(f"{path}: no word-embedding table among keys {sorted(obj)[:8]}")
    if obj.dim() != 2 or obj.shape[1] != sat_amd.Decoder.BERT_HIDDEN:
        raise ValueError(f"{path}: expected a [V, 768] table, got {tuple(obj.shape)}")
    return obj.float()


def build(args, device):
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    word_dict = None
    if args.bert:
        vocab = sat_amd.Decoder.BERT_VOCAB
    elif args.synthetic:   # generate_json_data.py:45-48 special ids + placeholder words
        vocab = args.vocab
        word_dict = {"<start>": 0, "<eos>": 1, "<unk>": 2, "<pad>": 3}
        word_dict.update({f"w{i}": i for i in range(4, vocab)})
    else:
        word_dict = json.load(open(os.path.join(args.data, "word_dict.json")))
        vocab = len(word_dict)
    encoder = sat_amd.Encoder(args.network, dtype=dt)
    if args.encoder_weights:
        encoder.load_state_dict(torch.load(args.encoder_weights, map_location="cpu", weights_only=True))
    bert_w = None
    if args.bert:
        if args.bert_embeddings:
            bert_w = load_bert_embeddings(args.bert_embeddings)
            vocab = bert_w.shape[0]
        elif not args.model:
            print("WARNING: --bert without --bert-embeddings or --model: the frozen word-embedding table is "
                  "randomly initialised, not bert-base-uncased's (decoder.py:21-36); this is not the reference's "
                  "BERT configuration", file=sys.stderr, flush=True)
    decoder = sat_amd.Decoder(vocab, encoder.dim, tf=args.tf, ado=args.ado, bert=args.bert, attention=args.attention,
                              bert_embedding_weight=bert_w)
    if args.model:   # train.py:65-67 (reference checkpoints load unchanged)
        decoder.load_state_dict(torch.load(args.model, map_location="cpu", weights_only=True))
    return encoder.to(device).eval(), decoder.to(device), word_dict, dt


SPLIT_SEED = {"train": 0, "val": 1, "test": 2}   # fixed per-split offsets (str hash() is randomised per process)


class ShardSampler(torch.utils.data.Sampler):
    """Rank r's items r, r+N, r+2N, ... of an evaluation split: every item exactly once across ranks
    (DistributedSampler pads with repeats), so gathered BLEU / meters cover the whole split."""

    def __init__(self, n, rank, world):
        self.idx = list(range(rank, n, world))

    def __iter__(self):
        return iter(self.idx)

    def __len__(self):
        return len(self.idx)


def loaders(args, split, rank, world):
    if args.synthetic:
        ds = SyntheticDataset(args.synthetic if split == "train" else max(args.batch_size, args.synthetic // 8),
                              args.vocab if not args.bert else sat_amd.Decoder.BERT_VOCAB,
                              32 if args.bert else args.seq, args.bert, seed=args.seed * 10 + SPLIT_SEED[split])
    else:
        ds = JsonCaptionDataset(args.data, split, args.fraction, args.bert, decode_only=not args.host_preprocess)
    train = split == "train"
    packed = not args.synthetic and not args.host_preprocess
    if world > 1:
        sampler = torch.utils.data.distributed.DistributedSampler(ds, world, rank, shuffle=True, seed=args.seed) \
            if train else ShardSampler(len(ds), rank, world)
    else:
        sampler = None
    # train.py:76-88: the reference shuffles train only and keeps every validation / test batch
    return torch.utils.data.DataLoader(ds, batch_size=args.batch_size, shuffle=train and sampler is None,
                                       sampler=sampler, num_workers=args.workers if not args.synthetic else 0,
                                       pin_memory=True, drop_last=train,
                                       collate_fn=sat_amd.collate_packed if packed else None)


def encoded_batches(loader, encoder, device, dt, max_steps, overlap):
    """(batch_idx, features, captions) of every training batch.  With ``overlap`` the frozen
    encoder forward (and the host-to-device copy) of batch i+1 is issued on a side stream before
    batch i is handed out, so it runs on the GPU beside batch i's decoder step, all-reduce and
    Adam (the encoder reads no decoder parameter; train.py:29-31 freezes it for VGG19 and the
    reference never optimises ResNet152's)."""
    main = torch.cuda.current_stream(device)
    side = torch.cuda.Stream(device) if overlap else main

    def encode(imgs, captions):
        with torch.cuda.stream(side), torch.no_grad():
            imgs = imgs.to(device, non_blocking=True)   # a Tensor, or PackedImages (uint8, native size)
            captions = captions.to(device, non_blocking=True)
            feats = encoder(imgs, dtype=dt)
            ev = torch.cuda.Event()
            ev.record(side)
        return feats, captions, ev

    pending = None
    for batch_idx, (imgs, captions, _) in enumerate(loader):
        if max_steps and batch_idx >= max_steps:
            break
        nxt = encode(imgs, captions)
        if pending is not None:
            yield pending
        feats, caps, ev = nxt
        main.wait_event(ev)
        if side is not main:   # produced on the side stream, consumed on the main one
            feats.record_stream(main)
            caps.record_stream(main)
        pending = (batch_idx, feats, caps)
    if pending is not None:
        yield pending


def train_epoch(epoch, encoder, decoder, opt, loader, args, device, dt, world, log, grad_ar=None):
    """train.py:119-192.  ``grad_ar``: a sat_amd.distributed.GradAllReduce for DP (N > 1)."""
    encoder.eval()
    decoder.train()
    pad, skip = sat_amd.special_ids(args.bert)
    # the reference updates its meters every batch (train.py:179-181) with 4 host syncs per step; here
    # they accumulate on the device and are read once per log line
    meters = sat_amd.RunningMeters(device)
    for batch_idx, feats, captions in encoded_batches(loader, encoder, device, dt, args.max_steps,
                                                      not args.no_overlap):
        opt.zero_grad()
        preds, alphas = decoder(feats, captions)
        loss, metrics = sat_amd.caption_loss(preds, alphas, captions, args.alpha_c, pad, skip)
        loss.backward()   # with DP the head bucket's all-reduce starts inside it, beside BPTT
        if grad_ar is not None:
            grad_ar.wait()
        opt.step()
        meters.update(loss, metrics)
        if batch_idx % args.log_interval == 0:   # train.py:183-192
            m = meters.read()
            log(dict(epoch=epoch, batch=batch_idx, train_loss=m["loss"], train_top1_acc=m["top1"],
                     train_top5_acc=m["top5"], train_loss_raw=m["loss_val"], train_tokens=m["count"]))
    return meters.read()["loss"] if meters.last is not None else 0.0


def evaluate(epoch, encoder, decoder, loader, args, device, dt, word_dict, mode, log):
    """train.py:198-347 (teacher-forced greedy hypotheses, BLEU-1..4)."""
    encoder.eval()
    decoder.eval()
    pad, skip = sat_amd.special_ids(args.bert)
    losses, top1, top5 = AverageMeter(), AverageMeter(), AverageMeter()
    refs, hyps = [], []
    tok = decoder.tokenizer if args.bert else None
    inv = {i: w for w, i in word_dict.items()} if word_dict else None
    with torch.no_grad():
        for batch_idx, (imgs, captions, all_caps) in enumerate(loader):
            if args.max_steps and batch_idx >= args.max_steps:
                break
            imgs, captions = imgs.to(device), captions.to(device)   # Tensor or PackedImages
            preds, alphas = decoder(encoder(imgs, dtype=dt), captions)
            loss, metrics = sat_amd.caption_loss(preds, alphas, captions, args.alpha_c, pad, skip)
            m = sat_amd.StepMetrics(loss, metrics).values()
            n = m["caption_length"]
            losses.update(m["loss"], n); top1.update(m["acc1"], n); top5.update(m["acc5"], n)
            ids = preds.argmax(dim=2).cpu().tolist()
            if args.bert:
                dec = lambda c: bleu_mod.decode_bert(c, tok)  # noqa: E731
            elif word_dict:
                dec = lambda c: bleu_mod.decode_plain(c, word_dict, inv)  # noqa: E731
            else:
                dec = lambda c: [str(t) for t in c if t not in (0, 3)][:c.index(1) if 1 in c else None]  # noqa: E731
            refs += [[dec(c) for c in cs] for cs in all_caps.tolist()]
            hyps += [dec(c) for c in ids]
    sums = [losses.sum, top1.sum, top5.sum, losses.count]
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        # every rank evaluated a disjoint shard (ShardSampler): gather hypotheses, references and the
        # meters' sums so the logged BLEU-1..4 and averages cover the whole split
        parts = [None] * dist.get_world_size()
        dist.all_gather_object(parts, (refs, hyps, sums))
        refs = [r for p in parts for r in p[0]]
        hyps = [h for p in parts for h in p[1]]
        sums = [sum(p[2][i] for p in parts) for i in range(4)]
    n = sums[3]
    avg = [v / n if n else 0.0 for v in sums[:3]]
    b1, b2, b3, b4 = bleu_mod.bleu_1_to_4(refs, hyps)
    log({"epoch": epoch, f"{mode}_loss": avg[0], f"{mode}_top1_acc": avg[1], f"{mode}_top5_acc": avg[2],
         f"{mode}_bleu1": b1, f"{mode}_bleu2": b2, f"{mode}_bleu3": b3, f"{mode}_bleu4": b4})
    return b4


def main(argv=None):
    args = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    set_seed(args.seed)

    def log(rec):
        if rank == 0:
            print(json.dumps(rec), flush=True)

    encoder, decoder, word_dict, dt = build(args, device)
    decoder.record_tokens = False   # no fed-token record per training step
    if not args.no_overlap:   # the decoder shares the chip with the next batch's encoder (bench.py defaults)
        decoder.split_target = 128 if args.network == "vgg19" else (96 if args.batch_size > 64 else 64)   # as bench.py
        # no layer3 block fused: the unfused c2 / c3 half-image kernels leave CUs to the decoder
        # (profiles/r2_s62_sched.txt)
        encoder.fuse_blocks = False
    opt = sat_amd.Adam(decoder.parameters(), lr=args.lr)
    grad_ar = sat_dist.GradAllReduce(decoder) if world > 1 else None
    sched = torch.optim.lr_scheduler.StepLR(opt, args.step_size)
    train_loader = loaders(args, "train", rank, world)
    val_loader = loaders(args, "val", rank, world)
    os.makedirs(args.out, exist_ok=True)
    enc_path = os.path.join(args.out, f"encoder_{args.network}.pth")
    if rank == 0:   # the trunk this run uses, so generate_caption.py encodes with the same weights
        torch.save({k: v.detach().cpu() for k, v in encoder.state_dict().items()}, enc_path)
    for epoch in range(1, args.epochs + 1):
        t0 = time.time()
        if isinstance(getattr(train_loader, "sampler", None), torch.utils.data.distributed.DistributedSampler):
            train_loader.sampler.set_epoch(epoch)
        train_epoch(epoch, encoder, decoder, opt, train_loader, args, device, dt, world, log, grad_ar)
        evaluate(epoch, encoder, decoder, val_loader, args, device, dt, word_dict, "val", log)
        sched.step()
        if rank == 0:   # train.py:103-110
            torch.save(decoder.state_dict(), os.path.join(args.out, f"model_{args.network}_{epoch}.pth"))
            cfg = dict(vars(args))
            cfg["encoder_weights"] = os.path.abspath(enc_path)
            if args.synthetic and word_dict:   # generate_caption.py reads <data>/word_dict.json
                cfg["data"] = args.out
                with open(os.path.join(args.out, "word_dict.json"), "w") as f:
                    json.dump(word_dict, f)
            with open(os.path.join(args.out, "model_config.json"), "w") as f:
                json.dump(cfg, f)
        log({"epoch": epoch, "epoch_seconds": time.time() - t0})
    if args.perform_test:
        test_loader = loaders(args, "test", rank, world)
        evaluate(args.epochs, encoder, decoder, test_loader, args, device, dt, word_dict, "test", log)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
