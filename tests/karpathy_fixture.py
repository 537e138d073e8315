"""A tiny dataset in the reference's Karpathy-JSON layout (generate_json_data.py:45-78): PNG images
of assorted sizes, <split>_img_paths.json with one entry per caption, <split>_captions.json padded
to a common length, word_dict.json with the four special ids."""
import json
import os

import numpy as np

SIZES = [(480, 640), (333, 500), (500, 375), (224, 224), (150, 100), (427, 640)]
WORDS = ["a", "dog", "runs", "on", "the", "grass", "cat", "sits", "mat", "two", "birds", "fly"]


def make_fixture(root, sizes=SIZES, caps_per_image=2, max_len=8, seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    os.makedirs(root, exist_ok=True)
    word_dict = {w: i + 4 for i, w in enumerate(WORDS)}
    word_dict.update({"<start>": 0, "<eos>": 1, "<unk>": 2, "<pad>": 3})
    with open(os.path.join(root, "word_dict.json"), "w") as f:
        json.dump(word_dict, f)
    paths, arrays = [], []
    for i, (h, w) in enumerate(sizes):
        # smooth gradients + noise: exercises every resampling weight, like a photo would
        yy, xx = np.mgrid[0:h, 0:w]
        base = np.stack([(xx * 255 // max(w - 1, 1)), (yy * 255 // max(h - 1, 1)), ((xx + yy) * 3) % 256], -1)
        img = np.clip(base + rng.integers(-40, 41, (h, w, 3)), 0, 255).astype(np.uint8)
        p = os.path.join(root, f"img_{i}.png")
        Image.fromarray(img, "RGB").save(p)
        paths.append(p)
        arrays.append(img)
    for split, idx in (("train", range(len(sizes))), ("val", range(0, len(sizes), 2)), ("test", range(1, len(sizes), 2))):
        img_paths, captions = [], []
        for i in idx:
            for _ in range(caps_per_image):
                n = int(rng.integers(2, max_len + 1))
                toks = [word_dict[WORDS[j]] for j in rng.integers(0, len(WORDS), n)]
                captions.append([0] + toks + [1] + [3] * (max_len - n))
                img_paths.append(paths[i])
        with open(os.path.join(root, f"{split}_img_paths.json"), "w") as f:
            json.dump(img_paths, f)
        with open(os.path.join(root, f"{split}_captions.json"), "w") as f:
            json.dump(captions, f)
    return paths, arrays, word_dict
