"""Models: checkpoint contract (keys / shapes / dtypes), param counts, differential
forward against the reference model classes, losses vs reference utils."""
import random

import numpy as np
import pytest
import torch

from apex_amd.envs import make
from apex_amd.model import AQL, DuelingDQN, NoisyLinear
from apex_amd.models.dqn import env_spec

from . import refimport

ATARI_KEYS = [("features.0.weight", (32, 4, 8, 8)), ("features.0.bias", (32,)), ("features.2.weight", (64, 32, 4, 4)),
              ("features.2.bias", (64,)), ("features.4.weight", (64, 64, 3, 3)), ("features.4.bias", (64,)),
              ("advantage.0.weight", (128, 3136)), ("advantage.0.bias", (128,)), ("advantage.2.weight", (18, 128)),
              ("advantage.2.bias", (18,)), ("value.0.weight", (128, 3136)), ("value.0.bias", (128,)),
              ("value.2.weight", (1, 128)), ("value.2.bias", (1,))]


def test_dueling_state_dict_contract():
    m = DuelingDQN.from_shapes((4, 84, 84), 18)
    sd = m.state_dict()
    assert [(k, tuple(v.shape)) for k, v in sd.items()] == ATARI_KEYS
    assert all(v.dtype == torch.float32 for v in sd.values())
    assert sum(p.numel() for p in m.parameters()) == 883_507
    assert sum(p.numel() for p in DuelingDQN.from_shapes((4, 84, 84), 6).parameters()) == 881_959
    assert sum(p.numel() for p in DuelingDQN(make("CartPole-v0")).parameters()) == 34_051


def test_flat_parameters_keep_state_dict(tmp_path):
    m = DuelingDQN.from_shapes((4, 84, 84), 6)
    before = {k: v.clone() for k, v in m.state_dict().items()}
    flat = m.flatten_parameters()
    assert flat.numel() == 881_959
    for k, v in m.state_dict().items():
        assert torch.equal(v, before[k])
    flat.add_(1.0)
    assert torch.equal(m.features[0].bias, before["features.0.bias"] + 1)
    torch.save(m.state_dict(), tmp_path / "model.pth")
    m2 = DuelingDQN.from_shapes((4, 84, 84), 6)
    m2.load_state_dict(torch.load(tmp_path / "model.pth", weights_only=True))
    x = torch.rand(2, 4, 84, 84) * 255
    torch.testing.assert_close(m(x), m2(x))


def test_aql_param_counts_and_keys():
    aql = AQL(make("CartPole-v0"), propose_sample=1, uniform_sample=50, device="cpu")
    assert aql.total_sample == 3 and sum(p.numel() for p in aql.parameters()) == 38_660
    keys = list(aql.state_dict())
    assert "q.advantage1.weight_epsilon" in keys and "proposal.dist_feature.2.bias" in keys
    bip = AQL(make("BipedalWalker-v3"), propose_sample=1, uniform_sample=50, device="cpu")
    assert bip.total_sample == 51 and sum(p.numel() for p in bip.parameters()) == 51_526
    a, a_mu, q = bip.act(make("BipedalWalker-v3").reset(), 0.0)
    assert a_mu.shape == (1, 51, 4) and q.shape == (1, 51)


@pytest.mark.skipif(not refimport.available(), reason="reference not mounted")
def test_dueling_forward_matches_reference_model():
    ref = refimport.load("model")
    env = env_spec((4, 84, 84), 18)
    theirs = ref.DuelingDQN(env)
    ours = DuelingDQN(env)
    ours.load_state_dict(theirs.state_dict())  # their checkpoint loads into ours
    theirs.load_state_dict(ours.state_dict())  # and vice versa
    x = torch.randint(0, 256, (3, 4, 84, 84)).float()
    torch.testing.assert_close(ours(x), theirs(x))
    random.seed(0)
    a1 = ours.act(x[0], 0.3)
    random.seed(0)
    a2 = theirs.act(x[0], 0.3)
    assert a1[0] == a2[0]
    np.testing.assert_allclose(a1[1], a2[1])


@pytest.mark.skipif(not refimport.available(), reason="reference not mounted")
def test_aql_forward_matches_reference_model():
    ref = refimport.load("model")
    for env_id in ("CartPole-v0", "BipedalWalker-v3"):
        env = make(env_id)
        torch.manual_seed(0)
        theirs = ref.AQL(env, propose_sample=2, uniform_sample=5, device="cpu")
        ours = AQL(env, propose_sample=2, uniform_sample=5, device="cpu")
        ours.load_state_dict(theirs.state_dict())
        s = env.reset()
        torch.manual_seed(7)
        np.random.seed(7)
        random.seed(7)
        r1 = theirs.act(s, 0.0)
        torch.manual_seed(7)
        np.random.seed(7)
        random.seed(7)
        r2 = ours.act(s, 0.0)
        assert int(r1[0]) == int(r2[0])
        np.testing.assert_allclose(r1[1], r2[1])
        torch.testing.assert_close(r1[2], r2[2])


@pytest.mark.skipif(not refimport.available(), reason="reference not mounted")
def test_compute_loss_matches_reference_utils():
    ref_utils = refimport.load("utils")
    from apex_amd import utils

    env = make("CartPole-v0")
    torch.manual_seed(0)
    model, tgt = DuelingDQN(env), DuelingDQN(env)
    B = 32
    g = torch.Generator().manual_seed(1)
    batch = (torch.randn(B, 4, generator=g), torch.randint(0, 2, (B,), generator=g), torch.randn(B, generator=g),
             torch.randn(B, 4, generator=g), (torch.rand(B, generator=g) < 0.2).float(), torch.rand(B, generator=g))
    l1, p1 = utils.compute_loss(model, tgt, batch, 3, 0.99)
    l2, p2 = ref_utils.compute_loss(model, tgt, batch, 3, 0.99)
    torch.testing.assert_close(l1, l2)
    np.testing.assert_allclose(p1, p2, rtol=1e-6)
    opt1 = torch.optim.RMSprop(model.parameters(), 1e-3, alpha=0.95, eps=1.5e-7, centered=True)
    model2 = DuelingDQN(env)
    model2.load_state_dict(model.state_dict())
    opt2 = torch.optim.RMSprop(model2.parameters(), 1e-3, alpha=0.95, eps=1.5e-7, centered=True)
    n1 = utils.update_parameters(l1, model, opt1, 40)
    l2b, _ = ref_utils.compute_loss(model2, tgt, batch, 3, 0.99)
    n2 = ref_utils.update_parameters(l2b, model2, opt2, 40)
    torch.testing.assert_close(torch.as_tensor(n1), torch.as_tensor(n2))
    for a, b in zip(model.parameters(), model2.parameters()):
        torch.testing.assert_close(a, b)


def test_noisy_linear_modes():
    torch.manual_seed(0)
    nl = NoisyLinear(8, 4, device="cpu")
    x = torch.randn(3, 8)
    nl.train()
    y1 = nl(x)
    nl.reset_noise()
    y2 = nl(x)
    assert not torch.allclose(y1, y2)
    nl.eval()
    torch.testing.assert_close(nl(x), torch.nn.functional.linear(x, nl.weight_mu, nl.bias_mu))
    assert set(nl.state_dict()) == {"weight_mu", "weight_sigma", "weight_epsilon", "bias_mu", "bias_sigma",
                                    "bias_epsilon"}
