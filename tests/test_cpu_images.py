"""Streaming image input, host side (no GPU): the oracle restatement of Pillow's 8-bit bilinear
resize is pinned bit-exact against PIL itself, the reference transform (train.py:27-32) against the
host-preprocess dataset path, and the decode-only dataset + PackedImages collate against the
Karpathy-layout fixture."""
import os
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import pil_resize as PR  # noqa: E402
from tests.karpathy_fixture import make_fixture  # noqa: E402

Image = pytest.importorskip("PIL.Image")


@pytest.mark.parametrize("h,w", [(480, 640), (333, 500), (224, 224), (150, 100), (1000, 231), (225, 223),
                                 (7, 3000)])
def test_oracle_resize_matches_pil(h, w):
    rng = np.random.default_rng(h * 7 + w)
    img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    ref = np.asarray(Image.fromarray(img, "RGB").resize((224, 224), Image.BILINEAR))
    got = PR.resize_bilinear(img, (224, 224))
    assert got.dtype == np.uint8 and got.shape == (224, 224, 3)
    assert np.array_equal(got, ref)


def test_oracle_resize_non_square_target():
    img = np.random.default_rng(1).integers(0, 256, (300, 410, 3), dtype=np.uint8)
    ref = np.asarray(Image.fromarray(img, "RGB").resize((96, 128), Image.BILINEAR))   # (W, H)
    assert np.array_equal(PR.resize_bilinear(img, (128, 96)), ref)


def test_oracle_transform_matches_host_dataset(tmp_path):
    import sat_amd  # noqa: F401
    from sat_amd import train as T
    paths, arrays, _ = make_fixture(str(tmp_path))
    ds = T.JsonCaptionDataset(str(tmp_path), "train")
    for i in range(0, len(ds), 2):
        x, cap, allc = ds[i]
        j = paths.index(ds.paths[i])
        assert np.array_equal(x.numpy(), PR.transform(arrays[j]))   # bit-identical fp32
        assert cap.shape == (10,) and allc.shape == (2, 10)


def test_decode_only_dataset_and_packed_collate(tmp_path):
    import sat_amd
    from sat_amd import train as T
    paths, arrays, _ = make_fixture(str(tmp_path))
    ds = T.JsonCaptionDataset(str(tmp_path), "train", decode_only=True)
    assert len(ds) == 12   # one entry per caption (dataset.py:27-38)
    items = [ds[i] for i in range(5)]
    for it in items:
        assert it[0].dtype == np.uint8 and it[0].ndim == 3 and it[0].shape[2] == 3
    packed, caps, allc = sat_amd.collate_packed(items)
    assert packed.count == 5 and caps.shape == (5, 10) and allc.shape == (5, 2, 10)
    assert packed.max_h == max(it[0].shape[0] for it in items)
    for b, it in enumerate(items):
        h, w = packed.sizes[b].tolist()
        o = int(packed.offsets[b])
        assert (h, w) == it[0].shape[:2]
        assert torch.equal(packed.pixels[o:o + h * w * 3], torch.from_numpy(it[0].reshape(-1)))
    assert int(packed.offsets[-1]) + int(packed.sizes[-1].prod()) * 3 == packed.pixels.numel()


def test_packed_images_validation():
    import sat_amd
    with pytest.raises(ValueError):
        sat_amd.PackedImages.from_arrays([])
    with pytest.raises(ValueError):
        sat_amd.PackedImages.from_arrays([np.zeros((4, 4), np.uint8)])
    with pytest.raises(ValueError):
        sat_amd.PackedImages.from_arrays([np.zeros((4, 4, 3), np.float32)])


def test_cli_parses_streaming_flags():
    from sat_amd import train as T
    a = T.parse(["--data", "x"])
    assert not a.host_preprocess and a.workers == 8
    a = T.parse(["--data", "x", "--host-preprocess", "--workers", "2"])
    assert a.host_preprocess and a.workers == 2
