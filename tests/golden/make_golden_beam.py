"""Golden vectors for beam-search captioning, from the REFERENCE ``Decoder.caption``
(decoder.py:160-269) run in the build container (see make_golden.py for the import rules:
read-only, no bytecode, ``mps_device`` -> CPU, BERT classes stubbed).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_beam.py

Weights come from ``oracle.sat_oracle.make_decoder_params`` (seeded, scaled by ``scale`` so
sentences run longer), with the end-token logit biased by ``eos_bias`` so beams retire at
different steps (a large negative bias exercises the "no completed sentence" exit after 51
steps).  Each npz holds the features of one image (expanded to beam rows at use, as
generate_caption.py:87 does), the returned sentence and alpha rows, and the
winning score (the oracle restatement is asserted equal to the reference while generating).
"""
import json
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)
from oracle import sat_oracle as O  # noqa: E402
from make_golden import import_reference, patch_bert  # noqa: E402

CONFIGS = [
    # name,              ado,   att,   bert,  beam, L,  D,  V,   eos ids,  eos_bias, weight scale
    ("att_simple_b3",    False, True,  False, 3,    16, 64, 60,  (1,),     0.0,  4.0),
    ("att_ado_b5",       True,  True,  False, 5,    16, 64, 60,  (1,),     0.5,  1.0),
    ("noatt_simple_b4",  False, False, False, 4,    12, 48, 50,  (1,),     1.0,  4.0),
    ("att_simple_b1",    False, True,  False, 1,    16, 64, 60,  (1,),     0.0,  4.0),
    ("att_simple_noend", False, True,  False, 3,    16, 64, 60,  (1, 102), -60.0, 1.0),
    ("bert_att_ado_b3",  True,  True,  True,  3,    16, 32, 128, (1, 0),   1.0,  1.0),
]


def main():
    ref_decoder = import_reference()
    torch.manual_seed(0)
    for (name, ado, att, bert, beam, L, D, V, eos_ids, eos_bias, scale) in CONFIGS:
        if bert:
            patch_bert(V)
        E = 768 if bert else 512
        seed = 31 + len(name)
        params = O.make_decoder_params(V, D, E, ado, seed, scale=scale)
        head_b = "f_out.bias" if ado else "deep_output.bias"
        for i in eos_ids:
            if i < V:
                params[head_b][i] += eos_bias
        dec = ref_decoder.Decoder(V, D, tf=False, ado=ado, bert=bert, attention=att)
        dec.load_state_dict(params, strict=True)
        dec.eval()
        rng = np.random.default_rng(seed + 1)
        one = torch.from_numpy(rng.standard_normal((1, L, D)).astype(np.float32))
        feats = one.expand(beam, L, D)
        with torch.no_grad():
            sentence, alpha = dec.caption(feats, beam)
        alpha = alpha.tolist() if torch.is_tensor(alpha) else alpha
        with torch.no_grad():
            ids, al, score = O.beam_search(params, feats.contiguous(), beam, ado=ado, attention=att, bert=bert)
        assert ids == sentence, (name, ids, sentence)
        np.testing.assert_allclose(np.array(al, dtype=np.float32), np.array(alpha, dtype=np.float32), rtol=1e-5,
                                   atol=1e-6)
        out = {"meta": np.array(json.dumps(dict(name=name, ado=ado, attention=att, bert=bert, beam=beam, L=L, D=D,
                                                V=V, E=E, seed=seed, eos_ids=list(eos_ids), eos_bias=eos_bias,
                                                scale=scale))),
               "img_features": one.numpy(), "sentence": np.array(sentence, dtype=np.int64),
               "alphas": np.array(alpha, dtype=np.float32), "score": np.float64(score)}
        path = os.path.join(HERE, f"beam_{name}.npz")
        np.savez_compressed(path, **out)
        print(f"{path}: len={len(sentence)} score={score:.4f} sentence={sentence[:12]}")


if __name__ == "__main__":
    main()
