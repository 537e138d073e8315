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


def beam_paths():
    return sorted(glob.glob(os.path.join(GOLDEN, "beam_*.npz")))


def beam_ids():
    return [os.path.basename(p)[len("beam_"):-4] for p in beam_paths()]


def load_beam(path):
    """Beam fixture (make_golden_beam.py) + its regenerated weights (end-token bias applied)."""
    from oracle import sat_oracle as O
    z = np.load(path, allow_pickle=False)
    d = {k: z[k] for k in z.files}
    cfg = d["cfg"] = json.loads(str(d["meta"]))
    p = O.make_decoder_params(cfg["V"], cfg["D"], cfg["E"], cfg["ado"], cfg["seed"], scale=cfg["scale"])
    head_b = "f_out.bias" if cfg["ado"] else "deep_output.bias"
    for i in cfg["eos_ids"]:
        if i < cfg["V"]:
            p[head_b][i] += cfg["eos_bias"]
    d["params"] = p
    d["feats"] = torch.from_numpy(d["img_features"]).expand(cfg["beam"], cfg["L"], cfg["D"]).contiguous()
    return d
