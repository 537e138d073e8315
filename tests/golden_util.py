"""Helpers to read the golden fixtures written by tests/golden/make_golden.py."""
import glob
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fixture_paths():
    return sorted(glob.glob(os.path.join(GOLDEN, "decoder_*.npz")))


def load(path):
    z = np.load(path, allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["cfg"] = json.loads(str(d["meta"]))
    d["grad_names"] = json.loads(str(d["grad_names"]))
    return d


def fixture_ids():
    return [os.path.basename(p)[len("decoder_"):-4] for p in fixture_paths()]


def params_for(cfg):
    from oracle import sat_oracle as O
    return O.make_decoder_params(cfg["V"], cfg["D"], cfg["E"], cfg["ado"], cfg["seed"])


def masks_for(cfg):
    from oracle import sat_oracle as O
    return O.make_dropout_masks(cfg["B"], cfg["T"] - 1, cfg["E"], cfg["seed"] + 3)


def t(x):
    return torch.from_numpy(np.asarray(x))
