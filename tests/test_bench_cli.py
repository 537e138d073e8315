"""bench.py host logic on CPU: argument modes for the BASELINE configs and the conv-launch
inventory the roofline is computed from (no GPU calls)."""
import sys

import pytest
import torch

import bench
from sat_amd.data import synthetic_captions


def _parse(monkeypatch, *argv):
    monkeypatch.setattr(sys, "argv", ["bench.py", *argv])
    return bench.parse()


def test_default_mode_is_the_metric_config(monkeypatch):
    a = _parse(monkeypatch)
    assert (a.gpus, a.batch, a.network, a.vocab, a.seq) == (1, 128, "resnet152", 10000, 27)
    assert not a.no_tf and not a.bert and not a.no_cpu_baseline


def test_bert_mode_uses_bert_vocabulary_and_slots(monkeypatch):
    # cfg5: BertConfig() vocabulary, [CLS] + 30 + [SEP] (generate_json_data_bert.py:47,69)
    a = _parse(monkeypatch, "--bert", "--network", "vgg19")
    assert (a.vocab, a.seq, a.network) == (30522, 32, "vgg19")
    assert a.no_cpu_baseline
    a = _parse(monkeypatch, "--bert", "--seq", "20")
    assert a.seq == 20


def test_no_tf_mode(monkeypatch):
    a = _parse(monkeypatch, "--no-tf")
    assert a.no_tf and a.vocab == 10000 and a.seq == 27


@pytest.mark.parametrize("network,n", [("resnet152", 155), ("vgg19", 16)])
def test_conv_launch_inventory(network, n):
    launches = bench.conv_launches(network, 1)
    assert len(launches) == n


def test_bert_synthetic_captions_layout():
    g = torch.Generator().manual_seed(0)
    caps = synthetic_captions(4, 32, 30522, generator=g, bert=True)
    assert caps.shape == (4, 32)
    assert (caps[:, 0] == 101).all() and (caps[:, -1] == 102).all()
    body = caps[:, 1:-1]
    assert ((body == 0) | ((body >= 1000) & (body < 30522))).all()
