"""Corpus BLEU as the reference computes it (train.py:330-333 -> nltk 3.8.1 corpus_bleu).

nltk is not in this image, so its published algorithm is restated here (nltk 3.8.1,
``nltk/translate/bleu_score.py``; default ``SmoothingFunction().method0``,
``auto_reweigh=False``):

  * per order n: clipped n-gram matches and hypothesis n-gram counts are summed over the
    corpus (modified precision numerator / max(1, denominator) per sentence);
  * brevity penalty from the summed closest-reference lengths (ties -> shorter) against the
    summed hypothesis lengths: 1 if hyp > ref, 0 if hyp == 0, else exp(1 - ref/hyp);
  * 0 is returned when there is no unigram match at all;
  * method0 replaces a zero precision by ``sys.float_info.min``;
  * score = BP * exp(fsum(w_n * log p_n)).

BLEU is host-side token bookkeeping (no GPU work): the decoder's greedy ids come off the
device once per evaluation batch.  Parity is exact by construction when ids are equal.
"""
import math
import sys
from collections import Counter


def _ngram_counts(tokens, n):
    return Counter(zip(*(tokens[i:] for i in range(n)))) if len(tokens) >= n else Counter()


def corpus_bleu(list_of_references, hypotheses, weights=(0.25, 0.25, 0.25, 0.25)):
    """nltk.translate.bleu_score.corpus_bleu (3.8.1 semantics, single weight tuple)."""
    if len(list_of_references) != len(hypotheses):
        raise ValueError("The number of hypotheses and their reference(s) should be the same")
    orders = len(weights)
    num = [0] * (orders + 1)
    den = [0] * (orders + 1)
    hyp_len_total = ref_len_total = 0
    for refs, hyp in zip(list_of_references, hypotheses):
        hyp = list(hyp)
        for n in range(1, orders + 1):
            h = _ngram_counts(hyp, n)
            if h:
                ref_max = Counter()
                for r in refs:
                    for ng, c in _ngram_counts(list(r), n).items():
                        if c > ref_max[ng]:
                            ref_max[ng] = c
                num[n] += sum(min(c, ref_max[ng]) for ng, c in h.items())
            den[n] += max(1, sum(h.values()))
        hl = len(hyp)
        hyp_len_total += hl
        ref_len_total += min((len(r) for r in refs), key=lambda rl: (abs(rl - hl), rl))
    if num[1] == 0:
        return 0
    if hyp_len_total > ref_len_total:
        bp = 1.0
    elif hyp_len_total == 0:
        bp = 0.0
    else:
        bp = math.exp(1 - ref_len_total / hyp_len_total)
    terms = []
    for n in range(1, orders + 1):
        p = num[n] / den[n] if num[n] else sys.float_info.min
        terms.append(weights[n - 1] * math.log(p))
    return bp * math.exp(math.fsum(terms))


def bleu_1_to_4(list_of_references, hypotheses):
    """The four scores run_evaluation logs (train.py:330-333), incl. BLEU-3's (0.33, 0.33, 0.33, 0)."""
    return (corpus_bleu(list_of_references, hypotheses, weights=(1, 0, 0, 0)),
            corpus_bleu(list_of_references, hypotheses, weights=(0.5, 0.5, 0, 0)),
            corpus_bleu(list_of_references, hypotheses, weights=(0.33, 0.33, 0.33, 0)),
            corpus_bleu(list_of_references, hypotheses))


def decode_plain(ids, word_dict, token_dict=None):
    """vanilla_decode_caption (train.py:277-285): stop at <eos>, drop <start>/<pad>."""
    token_dict = token_dict or {i: w for w, i in word_dict.items()}
    out = []
    for i in ids:
        if i == word_dict["<eos>"]:
            break
        if i not in (word_dict["<start>"], word_dict["<pad>"]):
            out.append(token_dict.get(i, "<unk>"))
    return out


def decode_bert(ids, tokenizer):
    """bert_decode_caption (train.py:250-260): stop at [SEP], drop [CLS]/[PAD]."""
    toks = tokenizer.convert_ids_to_tokens(ids)
    sent = []
    for t in toks:
        if t == "[SEP]":
            break
        if t not in ("[CLS]", "[PAD]"):
            sent.append(t)
    return tokenizer.convert_tokens_to_string(sent).split()
