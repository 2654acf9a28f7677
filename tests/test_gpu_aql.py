"""AQL HIP kernels (candidate critic, proposal sampling, selection) vs PyTorch fp32."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(env_id, dev, propose, uniform, seed=0):
    from apex_amd import envs
    from apex_amd.models.aql import AQL

    torch.manual_seed(seed)
    env = envs.make(env_id)
    m = AQL(env, propose_sample=propose, uniform_sample=uniform, device=dev).to(dev)
    with torch.no_grad():  # non-zero biases so every bias path is exercised
        for p in m.parameters():
            if p.dim() == 1:
                p.uniform_(-0.2, 0.2)
    return m, env


@pytest.mark.parametrize("env_id,propose,uniform", [("BipedalWalker-v3", 11, 13), ("Pendulum-v0", 5, 7),
                                                    ("CartPole-v0", 1, 50)])
@pytest.mark.parametrize("train", [True, False])
def test_candidate_q_matches_torch(cuda, env_id, propose, uniform, train):
    from apex_amd.models.aql_fused import FusedAQL

    m, env = _model(env_id, cuda, propose, uniform)
    m.train(train)
    f = FusedAQL(m)
    B = 37
    g = torch.Generator().manual_seed(1)
    st = torch.randn(B, m.input_shape[0], generator=g).to(cuda)
    if m.env_iscontinuous:
        am = torch.rand(B, m.total_sample, m.num_actions, generator=g).to(cuda) * 2 - 1
    else:
        am = torch.randint(0, m.num_actions, (B, m.total_sample), generator=g).float().to(cuda)
    with torch.no_grad():
        ref = m.q.candidate_q(st, am)
    got = f.candidate_q(st, am)
    torch.testing.assert_close(got, ref, rtol=2e-5, atol=2e-5)


def test_propose_continuous_distribution(cuda):
    from apex_amd.models.aql_fused import FusedAQL

    m, env = _model("BipedalWalker-v3", cuda, propose=64, uniform=64)
    f = FusedAQL(m)
    B = 512
    st = torch.randn(B, 24, device=cuda)
    am = f.propose(st)
    assert am.shape == (B, 128, 4)
    uni, prop = am[:, :64], am[:, 64:]
    assert float(uni.min()) >= -1.0 and float(uni.max()) <= 1.0
    assert abs(float(uni.mean())) < 0.02 and abs(float(uni.var()) - 1 / 3) < 0.02
    with torch.no_grad():
        mu = m.proposal.dist_feature(m.q.embedding_feature(st))
    z = (prop - mu[:, None, :]) / 0.5  # action_var 0.25 -> std 0.5
    assert abs(float(z.mean())) < 0.02 and abs(float(z.std()) - 1.0) < 0.02
    am2 = f.propose(st)  # counter advanced: fresh samples
    assert not torch.equal(am, am2)


def test_propose_discrete_without_replacement_and_categorical(cuda):
    from apex_amd.models.aql_fused import FusedAQL

    m, env = _model("MountainCar-v0", cuda, propose=40, uniform=3)
    f = FusedAQL(m)
    B = 2048
    st = torch.randn(B, 2, device=cuda)
    am = f.propose(st)
    assert am.shape == (B, 43)
    uni = am[:, :3].long()
    assert torch.equal(uni.sort(1).values, torch.arange(3, device=cuda).expand(B, 3))  # a permutation per row
    with torch.no_grad():
        p = torch.softmax(m.proposal.dist_feature(m.q.embedding_feature(st)), 1)
    counts = torch.stack([(am[:, 3:] == k).float().mean(1) for k in range(3)], 1)
    assert float((counts.mean(0) - p.mean(0)).abs().max()) < 0.01


def test_act_greedy_and_random(cuda):
    from apex_amd.models.aql_fused import FusedAQL

    m, env = _model("Pendulum-v0", cuda, propose=9, uniform=9)
    f = FusedAQL(m)
    B = 300
    st = torch.randn(B, 3, device=cuda)
    idx, am, act = f.act(st, 0.0)
    q = f.candidate_q(st, am)
    assert torch.equal(idx.long(), q.argmax(1))
    torch.testing.assert_close(act, am[torch.arange(B), idx.long()])
    idx1, am1, _ = f.act(st, 1.0)  # always random: spread over candidates
    assert len(torch.unique(idx1)) > 10


def test_aql_trainers_on_gpu(cuda, tmp_path):
    """AQL.py / AQL_dis.py equivalents on the MI355X: fused no-grad critics in the loss and
    GPU-batched actors (FusedAQL.act) replacing the CPU worker processes."""
    from apex_amd.trainers.aql import train_AQL, train_AQL_dis
    from apex_amd.utils.tb import NullWriter

    t = train_AQL("Pendulum-v0", max_step=80, seed=0, save_dir=str(tmp_path), writer=NullWriter(), save_interval=1000,
                  device="cuda", propose_sample=8, uniform_sample=8)
    assert t.fused is not None
    t.train()
    d = train_AQL_dis("BipedalWalker-v3", max_step=2, save_dir=str(tmp_path), writer=NullWriter(), device="cuda",
                      batch_size=16, gpu_actors=6, max_episode_length=60)
    n_eps = d.train()
    assert n_eps == 12 and 0 < len(d.replay_buffer) <= 6 * 60 * 2 and d.learn_idx > 0
    assert all(torch.isfinite(p).all() for p in d.model.parameters())
