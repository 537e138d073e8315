"""CPU restatement of the reference's image transform -- TEST INFRASTRUCTURE ONLY (imported by
tests/ alone; the product path is csrc/images.hip behind sat_images_to_input).

The reference resizes with torchvision 0.16's transforms.Resize((224, 224)) on PIL images
(/root/reference/train.py:27-32), i.e. Pillow's Image.resize(..., BILINEAR) (Pillow 10.1.0 pinned in
/root/reference/requirements.txt), then ToTensor (/255) and Normalize(mean, std).  Pillow is a
third-party dependency absent from /root/reference; its published 8-bit resampler
(libImaging/Resample.c: precompute_coeffs, normalize_coeffs_8bpc, ImagingResampleHorizontal_8bpc,
ImagingResampleVertical_8bpc) is restated here with numpy integer arithmetic.  Parity is pinned
against the Pillow importable in this container and on the GPU box (12.2; the resampler is unchanged
since 10.1) by tests/test_cpu_images.py: bytes bit-identical for up-, down- and non-scaled sizes.
"""
import math

import numpy as np

PREC = 22                                   # PRECISION_BITS = 32 - 8 - 2
MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)   # train.py:27-32
STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


def coeffs(in_size, out_size):
    """precompute_coeffs (BILINEAR, support 1, box (0, in)) + normalize_coeffs_8bpc:
    (lo [out], n [out], k [out, ksize] int64 fixed point)."""
    scale = float(np.float32(in_size)) / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    lo = np.zeros(out_size, np.int64)
    n = np.zeros(out_size, np.int64)
    k = np.zeros((out_size, ksize), np.int64)
    for i in range(out_size):
        center = 0.0 + (i + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)   # C (int) cast truncates toward zero, as int()
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = []
        ww = 0.0
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            f = 1.0 - t if t < 1.0 else 0.0
            w.append(f)
            ww += f
        if ww != 0.0:
            w = [v / ww for v in w]
        for x, v in enumerate(w):
            k[i, x] = int(-0.5 + v * (1 << PREC)) if v < 0 else int(0.5 + v * (1 << PREC))
        lo[i], n[i] = xmin, xmax
    return lo, n, k


def _clip8(ss):
    return np.where(ss >= (1 << PREC << 8), 255, np.where(ss <= 0, 0, ss >> PREC)).astype(np.uint8)


def _pass(img, axis, out_size):
    """One resampling pass along ``axis`` (1 = horizontal, 0 = vertical) of an [H, W, 3] uint8 image."""
    lo, n, k = coeffs(img.shape[axis], out_size)
    idx = lo[:, None] + np.arange(k.shape[1])[None, :]                 # [out, ksize]
    idx = np.minimum(idx, img.shape[axis] - 1)                         # taps past n have k == 0
    src = img.astype(np.int64)
    if axis == 1:
        g = src[:, idx, :]                                             # [H, out, ksize, 3]
        ss = (1 << (PREC - 1)) + np.einsum("hokc,ok->hoc", g, k)
    else:
        g = src[idx, :, :]                                             # [out, ksize, W, 3]
        ss = (1 << (PREC - 1)) + np.einsum("okwc,ok->owc", g, k)
    return _clip8(ss)


def resize_bilinear(img, size):
    """Pillow Image.resize((W, H), BILINEAR) of an RGB [H, W, 3] uint8 array -> [OH, OW, 3] uint8
    (horizontal pass first, 8-bit intermediate, as ImagingResampleInner)."""
    OH, OW = size
    out = _pass(img, 1, OW)
    return _pass(out, 0, OH)


def transform(img, size=(224, 224)):
    """Resize -> ToTensor -> Normalize of one [H, W, 3] uint8 image: [3, OH, OW] float32."""
    r = resize_bilinear(img, size).astype(np.float32)
    x = (r / np.float32(255.0) - MEAN) / STD
    return np.ascontiguousarray(x.transpose(2, 0, 1))
