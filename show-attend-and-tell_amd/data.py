"""Synthetic inputs in the reference's data layout.

Images: the post-Normalize domain of train.py:27-32, i.e. [B,3,224,224] f32 ~ N(0,1).
Plain captions ``<start>=0 w.. <eos>=1 <pad>=3..`` (generate_json_data.py:71-78),
n ~ U{8..T-2}, words ~ U[4,V).  BERT captions ``[CLS]=101 w.. [PAD]=0.. [SEP]=102``
(generate_json_data_bert.py:44-47; SEP after the padding, as the reference writes it).

PackedImages: the streaming real-data input.  Host workers only decode
(dataset.py:9-12 pil_loader); the batch travels as uint8 HWC pixels at native size and
ops.images_to_input does Resize + ToTensor + Normalize (train.py:27-32) on the GPU.
"""
import numpy as np
import torch


def synthetic_captions(B, T, V, generator=None, bert=False, device="cpu"):
    g = generator
    body = T - 2
    if bert:
        n = torch.randint(1, body + 1, (B,), generator=g)
        words = torch.randint(min(1000, V - 1), V, (B, body), generator=g)
        pos = torch.arange(body).unsqueeze(0)
        body_t = torch.where(pos < n.unsqueeze(1), words, torch.zeros_like(words))
        caps = torch.cat([torch.full((B, 1), 101), body_t, torch.full((B, 1), 102)], 1)
    else:
        n = torch.randint(min(8, body), body + 1, (B,), generator=g)
        words = torch.randint(4, V, (B, body + 1), generator=g)
        pos = torch.arange(body + 1).unsqueeze(0)
        ln = n.unsqueeze(1)
        body_t = torch.where(pos < ln, words, torch.where(pos == ln, torch.ones_like(words), torch.full_like(words, 3)))
        caps = torch.cat([torch.zeros(B, 1, dtype=torch.long), body_t], 1)
    return caps.long().to(device)


def synthetic_images(B, H=224, W=224, generator=None, device="cpu"):
    return torch.randn(B, 3, H, W, generator=generator).to(device)


class PackedImages:
    """A batch of decoded RGB images of any sizes: ``pixels`` uint8 (all images HWC back to back),
    ``offsets`` int64 [B] (start of image b in pixels), ``sizes`` int32 [B, 2] = (H, W)."""

    def __init__(self, pixels, offsets, sizes, max_h, max_w):
        self.pixels, self.offsets, self.sizes = pixels, offsets, sizes
        self.max_h, self.max_w = int(max_h), int(max_w)

    @property
    def count(self):
        return int(self.offsets.shape[0])

    def __len__(self):
        return self.count

    @classmethod
    def from_arrays(cls, arrays):
        """[H, W, 3] uint8 arrays (np or torch) -> one packed host batch."""
        if not arrays:
            raise ValueError("PackedImages: empty batch")
        sizes, offsets, total = [], [], 0
        for a in arrays:
            if a.ndim != 3 or a.shape[2] != 3 or a.dtype not in (np.uint8, torch.uint8):
                raise ValueError(f"PackedImages: expected [H, W, 3] uint8 images, got {tuple(a.shape)} {a.dtype}")
            offsets.append(total)
            sizes.append((a.shape[0], a.shape[1]))
            total += a.shape[0] * a.shape[1] * 3
        pixels = torch.empty(total, dtype=torch.uint8)
        for a, o, (h, w) in zip(arrays, offsets, sizes):
            src = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.require(a, np.uint8, ["C", "W"]))
            pixels[o:o + h * w * 3] = src.reshape(-1)
        sz = torch.tensor(sizes, dtype=torch.int32)
        return cls(pixels, torch.tensor(offsets, dtype=torch.int64), sz, int(sz[:, 0].max()), int(sz[:, 1].max()))

    def pin_memory(self):   # torch DataLoader(pin_memory=True) hook
        return PackedImages(self.pixels.pin_memory(), self.offsets.pin_memory(), self.sizes.pin_memory(),
                            self.max_h, self.max_w)

    def to(self, device, non_blocking=False):
        return PackedImages(self.pixels.to(device, non_blocking=non_blocking),
                            self.offsets.to(device, non_blocking=non_blocking),
                            self.sizes.to(device, non_blocking=non_blocking), self.max_h, self.max_w)

    def record_stream(self, stream):
        for t in (self.pixels, self.offsets, self.sizes):
            t.record_stream(stream)


def collate_packed(batch):
    """DataLoader collate for (uint8 HWC image, caption, all captions) items."""
    imgs, caps, all_caps = zip(*batch)
    return (PackedImages.from_arrays(list(imgs)), torch.utils.data.default_collate(list(caps)),
            torch.utils.data.default_collate(list(all_caps)))
