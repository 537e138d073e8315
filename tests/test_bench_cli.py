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


@pytest.mark.parametrize("network,fused,fused2,n", [("resnet152", False, False, 155),
                                                    ("resnet152", True, False, 155 - 2 * 35),
                                                    ("resnet152", False, True, 155 - 2 * 7),
                                                    ("resnet152", True, True, 155 - 2 * 42),
                                                    ("vgg19", True, True, 16)])
def test_conv_launch_inventory(network, fused, fused2, n):
    launches = bench.conv_launches(network, 1, fused=fused, fused2=fused2)
    assert len(launches) == n
    blocks = [l for l in launches if l.get("fused")]
    nb3, nb2 = (35 if fused else 0), (7 if fused2 else 0)
    assert len(blocks) == (nb3 + nb2 if network == "resnet152" else 0)
    un = {l["cls"].split()[0]: l["flops"] for l in bench.conv_launches(network, 1, fused=False, fused2=False)}
    if network != "resnet152":
        return
    for li, nb in ((2, nb2), (3, nb3)):   # one fused block = c1 + c2 + c3 of the unfused inventory
        mine = [b for b in blocks if b["cls"].startswith(f"L{li}block")]
        assert len(mine) == nb
        if mine:
            assert abs(mine[0]["flops"] - (un[f"L{li}c1"] + un[f"L{li}c2"] + un[f"L{li}c3+res"])) < 1


def test_bert_synthetic_captions_layout():
    g = torch.Generator().manual_seed(0)
    caps = synthetic_captions(4, 32, 30522, generator=g, bert=True)
    assert caps.shape == (4, 32)
    assert (caps[:, 0] == 101).all() and (caps[:, -1] == 102).all()
    body = caps[:, 1:-1]
    assert ((body == 0) | ((body >= 1000) & (body < 30522))).all()


@pytest.mark.parametrize("args,gflop", [((49, 2048, 512, 10000, 27, True), 2.53),    # ResNet152 / V10k, ado
                                        ((196, 512, 512, 2600, 27, True), 1.20),     # VGG19 / Flickr8k
                                        ((196, 512, 768, 30522, 27, False), 5.30)])  # BERT, simple head
def test_decoder_flops_match_survey(args, gflop):
    """decoder fwd+bwd GFLOP/img with W.a hoisted (the whole-step roofline's decoder part)."""
    from sat_amd.diagnostics import decoder_flops
    assert abs(decoder_flops(*args[:5], ado=args[5]) / 1e9 - gflop) < 0.01


def test_step_group_bytes_bench_shape():
    """Per-step algorithmic bytes of the fused attention step at the bench shape (the
    attention forward streams Ws and the annotation vectors once: ~38 MB at B=128, L=49, D=2048, bf16)."""
    from sat_amd.diagnostics import step_group_bytes, GROUPS
    by = step_group_bytes(128, 49, 2048, 512, 27, 2)
    assert set(by) == set(GROUPS)
    assert 35e6 < by["attn_fwd"] < 40e6
    assert all(v > 0 for v in by.values())
    assert step_group_bytes(128, 49, 2048, 512, 27, 2, attention=False)["attn_fwd"] == 0


def test_bench_defaults_time_enough_steps(monkeypatch):
    a = _parse(monkeypatch)
    assert a.steps >= 200 and a.fp32_steps > 0


def test_gpus_flag_relaunches_as_ranks(monkeypatch):
    """`python bench.py --gpus N` (N > 1, not already a rank) starts N ranks through torch.distributed.run with the
    same arguments, on 127.0.0.1, and exits with their status; the parent touches no GPU."""
    calls = []

    class Done:
        returncode = 3

    def fake_run(cmd, env):
        calls.append((cmd, env))
        return Done()
    import subprocess
    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "7", "--dist-backend", "gloo"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 3
    (cmd, env), = calls
    i = cmd.index("-m")
    assert cmd[i + 1] == "torch.distributed.run"
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-5:] == ["--gpus", "8", "--steps", "7", "--dist-backend", "gloo"][-5:]
    assert cmd[cmd.index("--master-addr=127.0.0.1") + 2].endswith("bench.py")
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert not torch.cuda.is_initialized()


def test_rank_checks_world_size(monkeypatch):
    """A rank launched for --gpus 4 under a 2-rank torch.distributed.run refuses to measure."""
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.main()


def test_single_gpu_runs_in_process(monkeypatch):
    """--gpus 1 (the default) never relaunches."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "launch_ranks", lambda *a: pytest.fail("relaunched"))
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    monkeypatch.setattr(bench.torch.cuda, "set_device", lambda *a: (_ for _ in ()).throw(RuntimeError("stop")))
    with pytest.raises(RuntimeError, match="stop"):
        bench.main()


def test_dp_rehearse_flag(monkeypatch):
    """--dp-rehearse (N = 1): the data-parallel path over a one-rank process group, off by default."""
    assert _parse(monkeypatch).dp_rehearse is False
    a = _parse(monkeypatch, "--dp-rehearse")
    assert a.dp_rehearse is True and a.gpus == 1 and a.dist_backend == "nccl"
