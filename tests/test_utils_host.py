"""CPU tests for the small reference utilities and the
dependency-free TensorBoard writer."""
import random
import warnings

import numpy as np
import pytest
import torch


def test_set_global_seeds_and_print_args(capsys):
    import argparse

    from apex_amd.utils import print_args, set_global_seeds

    draws = []
    for _ in range(2):
        set_global_seeds(7, use_torch=True)
        draws.append((np.random.rand(), random.random(), torch.rand(1).item()))
    assert draws[0] == draws[1]
    print_args(argparse.Namespace(lr=1e-4, env="Pong"))
    out = capsys.readouterr().out.splitlines()
    assert out[0].strip() == "Options" and out[1].strip() == "lr: 0.0001" and out[2].strip() == "env: Pong"


def test_png_roundtrip():
    from apex_amd.utils import array2png, png2array

    a = np.random.default_rng(0).integers(0, 256, (84, 84), dtype=np.uint8)
    png = array2png(a)
    assert png[:8] == b"\x89PNG\r\n\x1a\n"
    assert np.array_equal(png2array(png), a)


def test_epsilon_ladder_and_single_actor():
    from apex_amd.algo.schedules import actor_epsilon, beta_by_frame, epsilon_by_frame

    # origin actor.py:69 -- eps_i = 0.4^(1 + 7 i/(N-1))
    ids = np.arange(8)
    eps = actor_epsilon(ids, 8)
    assert np.allclose(eps, 0.4 ** (1 + 7 * ids / 7))
    assert eps[0] == pytest.approx(0.4) and eps[-1] == pytest.approx(0.4 ** 8)
    assert np.all(np.diff(eps) < 0)
    # one actor divides by zero in the reference; here eps_0 = eps_base
    assert actor_epsilon(0, 1) == 0.4
    assert np.array_equal(actor_epsilon(np.zeros(3), 1), np.full(3, 0.4))
    assert beta_by_frame(0) == pytest.approx(0.4) and beta_by_frame(500) == pytest.approx(0.7)
    assert beta_by_frame(10 ** 6) == 1.0
    assert epsilon_by_frame(0) == pytest.approx(1.0)
    assert epsilon_by_frame(500) == pytest.approx(0.01 + 0.99 * np.exp(-1))


def test_scheduler_steps_before_optimizer():
    """the reference calls scheduler.step() before optimizer.step(), so the
    first update already runs at the decayed LR."""
    from apex_amd.algo.schedules import step_scheduler_early

    p = torch.nn.Parameter(torch.ones(1))
    opt = torch.optim.SGD([p], lr=1.0)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5)
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # the helper must silence torch's ordering warning itself
        step_scheduler_early(sched)
    p.grad = torch.ones(1)
    opt.step()
    assert p.item() == pytest.approx(0.5)  # 1 - 0.5 * 1


def test_summary_writer_event_file(tmp_path):
    import json

    from apex_amd.utils.tb import SummaryWriter, crc32c, read_records

    assert crc32c(b"123456789") == 0xE3069283  # CRC-32C check value
    w = SummaryWriter(str(tmp_path))
    w.add_scalar("loss", torch.tensor(1.5), 3)
    w.add_scalars("q", {"mean": 2.0, "max": 4.0}, 4)
    w.close()
    recs = read_records(w.event_path)  # asserts both crcs of every record
    assert len(recs) == 4
    assert b"brain.Event:2" in recs[0]
    assert b"loss" in recs[1] and b"q/mean" in recs[2] and b"q/max" in recs[3]
    rows = [json.loads(x) for x in open(tmp_path / "scalars.jsonl")]
    assert [(r["tag"], r["value"], r["step"]) for r in rows] == [("loss", 1.5, 3), ("q/mean", 2.0, 4),
                                                                ("q/max", 4.0, 4)]


def test_enjoy_plays_saved_checkpoint(tmp_path, capsys):
    from apex_amd.config import argparser
    from apex_amd.models.dqn import DuelingDQN
    from apex_amd.roles.common import make_role_env
    from apex_amd.roles.enjoy import main
    from apex_amd.utils.checkpoint import save_model

    cfg = argparser(["--env", "CartPole-v0"]).config
    path = save_model(DuelingDQN(make_role_env(cfg)), str(tmp_path / "model.pth"))
    res = main(["--env", "CartPole-v0", "--model", path, "--episodes", "2"])
    assert len(res) == 2 and all(n >= 1 and r == n for n, r in res)  # CartPole: +1 per step
    assert capsys.readouterr().out.count("Episode Length / Reward:") == 2


def test_engine_checkpoint_sidecar_tagged(tmp_path):
    """train.save_engine writes the sidecar atomically with a weights fingerprint; a
    sidecar from a different save (torn save) is ignored by load_engine."""
    import types
    import warnings

    import torch

    from apex_amd.models.dqn import DuelingDQN
    from apex_amd.train import load_engine, save_engine

    def learner(seed):
        torch.manual_seed(seed)
        m = DuelingDQN.from_shapes((4,), 3)
        flat = m.flatten_parameters()
        return types.SimpleNamespace(model=m, flat=flat, opt_s1=torch.rand_like(flat), opt_s2=torch.rand_like(flat),
                                     step_counter=torch.tensor([seed + 5]), tflat=flat.clone() + 1, hip_net=False)

    a = learner(1)
    path = str(tmp_path / "model.pth")
    save_engine(a, path, {"learn_steps": 7})
    b = learner(2)
    assert load_engine(b, path) == {"learn_steps": 7}
    assert torch.equal(b.flat, a.flat) and torch.equal(b.opt_s1, a.opt_s1) and int(b.step_counter) == 6
    # torn save: the model file is newer than the sidecar
    c = learner(3)
    torch.save({k: v.clone() for k, v in c.model.state_dict().items()}, path)
    d = learner(4)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert load_engine(d, path) == {}
    assert any("torn" in str(x.message) for x in w)
    assert torch.equal(d.flat, c.flat) and torch.equal(d.tflat, d.flat)
