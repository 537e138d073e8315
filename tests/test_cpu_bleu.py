"""BLEU (train.py:330-333 via nltk 3.8.1 corpus_bleu, restated -- nltk is not in the image).
Pinned by nltk's own published doctest values and hand-computed cases; the product
implementation (sat_amd.bleu) must equal the oracle restatement on random corpora."""
import math
import random

import pytest

import sat_amd.bleu as B
from oracle import sat_oracle as O

# nltk/translate/bleu_score.py docstring example (sentence_bleu / corpus_bleu doctests)
HYP1 = ['It', 'is', 'a', 'guide', 'to', 'action', 'which', 'ensures', 'that', 'the', 'military', 'always',
        'obeys', 'the', 'commands', 'of', 'the', 'party']
REF1A = ['It', 'is', 'a', 'guide', 'to', 'action', 'that', 'ensures', 'that', 'the', 'military', 'will',
         'forever', 'heed', 'Party', 'commands']
REF1B = ['It', 'is', 'the', 'guiding', 'principle', 'which', 'guarantees', 'the', 'military', 'forces', 'always',
         'being', 'under', 'the', 'command', 'of', 'the', 'Party']
REF1C = ['It', 'is', 'the', 'practical', 'guide', 'for', 'the', 'army', 'always', 'to', 'heed', 'the',
         'directions', 'of', 'the', 'party']
HYP2 = ['he', 'read', 'the', 'book', 'because', 'he', 'was', 'interested', 'in', 'world', 'history']
REF2A = ['he', 'was', 'interested', 'in', 'world', 'history', 'because', 'he', 'read', 'the', 'book']


@pytest.mark.parametrize("impl", [B.corpus_bleu, O.corpus_bleu])
def test_nltk_doctest_values(impl):
    assert impl([[REF1A, REF1B, REF1C]], [HYP1]) == pytest.approx(0.5045666840058485, abs=1e-12)
    assert impl([[REF1A, REF1B, REF1C], [REF2A]], [HYP1, HYP2]) == pytest.approx(0.5920778868801042, abs=1e-12)


@pytest.mark.parametrize("impl", [B.corpus_bleu, O.corpus_bleu])
def test_hand_computed(impl):
    assert impl([[list("abcd")]], [list("abcd")]) == pytest.approx(1.0)
    # p1 = 2/3, p2 = 1/2, BP = 1  ->  BLEU-2 = sqrt(1/3)
    assert impl([[list("abd")]], [list("abc")], weights=(0.5, 0.5, 0, 0)) == pytest.approx(math.sqrt(1 / 3))
    # brevity: hyp 2 vs ref 4 -> BP = e^-1, p1 = p2 = 1
    assert impl([[list("abcd")]], [list("ab")], weights=(0.5, 0.5, 0, 0)) == pytest.approx(math.exp(-1))
    # no unigram match -> exactly 0 ; empty hypothesis -> 0
    assert impl([[list("abc")]], [list("xyz")]) == 0
    assert impl([[list("abc")]], [[]]) == 0
    # a zero higher-order precision is replaced by float_info.min (method0): tiny but > 0
    v = impl([[list("abd")]], [list("abc")])
    assert 0 < v < 1e-100


def test_product_equals_oracle_on_random_corpora():
    rng = random.Random(0)
    vocab = [f"w{i}" for i in range(12)]
    for _ in range(50):
        refs, hyps = [], []
        for _ in range(rng.randint(1, 6)):
            refs.append([[rng.choice(vocab) for _ in range(rng.randint(0, 9))] for _ in range(rng.randint(1, 5))])
            hyps.append([rng.choice(vocab) for _ in range(rng.randint(0, 9))])
        for w in [(1, 0, 0, 0), (0.5, 0.5, 0, 0), (0.33, 0.33, 0.33, 0), (0.25, 0.25, 0.25, 0.25)]:
            assert B.corpus_bleu(refs, hyps, w) == O.corpus_bleu(refs, hyps, w)


def test_caption_decoding_rules():
    wd = {"<start>": 0, "<eos>": 1, "<unk>": 2, "<pad>": 3, "a": 4, "dog": 5}
    assert B.decode_plain([0, 4, 5, 1, 3, 3], wd) == ["a", "dog"]
    assert B.decode_plain([0, 3, 4, 3, 5], wd) == ["a", "dog"]
    from sat_amd.decoder import BertTokenizerStub
    tok = BertTokenizerStub()
    assert B.decode_bert([101, 2000, 0, 0, 102, 2001], tok) == ["tok2000"]
