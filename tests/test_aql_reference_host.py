"""AQL pinned to the reference itself (VERDICT r2 Next #6): with identical weights and an
identical sampled batch, one AQL_dis learner step of this framework
(``trainers.aql.aql_update`` -> ``algo.losses.compute_loss_AQL`` + ``Proposal_Network.evaluate``)
matches the reference's ``utils.compute_loss_AQL`` (utils.py:44-61) and its proposal loss /
update sequence (AQL_dis.py:63-108) built from the reference's own ``model.AQL``:
losses, priorities, every parameter gradient, the parameters after both Adam steps, the
proposal hard copy and the NoisyNet reset.  The GPU engine's fp64 test
(tests/test_gpu_aql_engine.py) compares against these same functions, so it is pinned
transitively."""
import numpy as np
import pytest
import torch

from apex_amd.envs import make
from apex_amd.model import AQL
from apex_amd.trainers.aql import aql_update

from . import refimport

pytestmark = pytest.mark.skipif(not refimport.available(), reason="reference not mounted")


def _batch(env, model, B, seed):
    g = torch.Generator().manual_seed(seed)
    obs = env.observation_space.shape[0]
    T = model.total_sample
    s = torch.randn(B, obs, generator=g)
    s2 = s + 0.1 * torch.randn(B, obs, generator=g)
    a = torch.randint(0, T, (B,), generator=g)
    r = torch.randn(B, generator=g)
    d = (torch.rand(B, generator=g) < 0.2).float()
    if model.env_iscontinuous:
        a_mu = torch.rand(B, T, model.num_actions, generator=g) * 2 - 1
    else:  # stored LongTensor candidates, read back through torch.FloatTensor (AQL_dis.py:73)
        a_mu = torch.stack([torch.randperm(model.num_actions, generator=g)[:T] if T <= model.num_actions
                            else torch.randint(0, model.num_actions, (T,), generator=g) for _ in range(B)]).float()
    w = torch.rand(B, generator=g) * 0.9 + 0.1
    return s, a, r, s2, d, a_mu, w


def _ref_td_step(ref_utils, model, target, opt_q, opt_p, batch, B, n_steps, gamma, ent_lam):
    """AQL_dis.py:63-108 (train_DQN.compute_td_loss after sampling), on reference objects."""
    state, action, reward, next_state, done, a_mu, weights = batch
    q_values = model(state, a_mu)
    embed_state = model.q.embedding_feature(state)
    dist = model.proposal.evaluate(embed_state)
    max_q_action = a_mu[torch.arange(B), q_values.max(1)[1]].reshape(B, -1)
    log_prob = dist.log_prob(max_q_action)
    entropy = dist.entropy()
    loss_p = torch.mean(-log_prob - ent_lam * entropy)
    opt_p.zero_grad()
    loss_p.backward()
    torch.nn.utils.clip_grad.clip_grad_norm_(model.proposal.parameters(), 40)
    opt_p.step()
    target.proposal.load_state_dict(model.proposal.state_dict())
    loss_q, prios = ref_utils.compute_loss_AQL(model, target, batch, n_steps=n_steps, gamma=gamma)
    opt_q.zero_grad()
    loss_q.backward()
    torch.nn.utils.clip_grad.clip_grad_norm_(model.q.parameters(), 40)
    opt_q.step()
    model.reset_noise()
    target.reset_noise()
    return loss_q, loss_p, prios


class _FixedBuffer:
    """Stands in for CustomPrioritizedReplayBuffer_AQL.sample/update_priorities with a fixed batch."""

    def __init__(self, batch):
        self.batch = batch
        self.prios = None

    def sample(self, batch_size, beta):
        s, a, r, s2, d, a_mu, w = self.batch
        return (s.numpy(), a.numpy(), r.numpy(), s2.numpy(), d.numpy(), a_mu.numpy(), w.numpy(),
                list(range(batch_size)))

    def update_priorities(self, idx, prios):
        self.prios = np.asarray(prios)


def _grads(m):
    return {n: (None if p.grad is None else p.grad.detach().clone()) for n, p in m.named_parameters()}


@pytest.mark.parametrize("env_id", ["CartPole-v0", "BipedalWalker-v3"])
def test_aql_dis_step_matches_reference(env_id):
    ref_model = refimport.load("model")
    ref_utils = refimport.load("utils")
    env = make(env_id)
    torch.manual_seed(3)
    theirs = ref_model.AQL(env, propose_sample=1, uniform_sample=50, device="cpu")
    theirs_t = ref_model.AQL(env, propose_sample=1, uniform_sample=50, device="cpu")
    theirs_t.load_state_dict(theirs.state_dict())
    ours = AQL(env, propose_sample=1, uniform_sample=50, device="cpu")
    ours_t = AQL(env, propose_sample=1, uniform_sample=50, device="cpu")
    ours.load_state_dict(theirs.state_dict())
    ours_t.load_state_dict(theirs_t.state_dict())
    assert list(ours.state_dict()) == list(theirs.state_dict())
    for m in (theirs, theirs_t, ours, ours_t):
        m.q.train()
    lr, B = 1e-3, 32
    opt_q_r = torch.optim.Adam(theirs.q.parameters(), lr)
    opt_p_r = torch.optim.Adam(theirs.proposal.parameters(), lr)
    opt_q_o = torch.optim.Adam(ours.q.parameters(), lr)
    opt_p_o = torch.optim.Adam(ours.proposal.parameters(), lr)
    for step in range(3):
        batch = _batch(env, ours, B, seed=100 + step)
        torch.manual_seed(50 + step)  # reset_noise draws from the torch RNG: same stream for both
        lq_r, lp_r, pr_r = _ref_td_step(ref_utils, theirs, theirs_t, opt_q_r, opt_p_r, batch, B, 1, 0.99, 0.8)
        g_r = _grads(theirs)
        buf = _FixedBuffer(batch)
        torch.manual_seed(50 + step)
        lq_o, lp_o = aql_update(ours, ours_t, buf, opt_q_o, opt_p_o, B, 0.4, 0.99, 1, 0.8, "cpu",
                                copy_proposal_to_target=True, reset_noise=True)
        g_o = _grads(ours)
        torch.testing.assert_close(lq_o, lq_r, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(lp_o, lp_r, rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(buf.prios, pr_r, rtol=1e-6, atol=1e-7)
        assert g_o.keys() == g_r.keys()
        for n in g_r:
            assert (g_o[n] is None) == (g_r[n] is None), n
            if g_r[n] is not None:
                torch.testing.assert_close(g_o[n], g_r[n], rtol=1e-5, atol=1e-7, msg=n)
        # Adam's first steps move a parameter by ~lr * g / (|g| + eps): for a gradient near 0 an
        # ulp-level gradient difference becomes a visible (but < 1 % of lr) parameter difference
        for m_o, m_r in ((ours, theirs), (ours_t, theirs_t)):
            for (n, a), b in zip(m_o.state_dict().items(), m_r.state_dict().values()):
                torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-2 * lr, msg=n)


def test_gpu_aql_engine_target_sync_cadence():
    """engine.aql.target_sync_due: the reference syncs after the SGD loop of every iteration
    whose index is a multiple of target_update_interval, iteration 0 included
    (AQL_dis.py:127-129); the learner-step cadence is opt-in."""
    from apex_amd.engine.aql import AQLEngineConfig, target_sync_due

    cfg = AQLEngineConfig()
    assert cfg.target_update_interval == 20 and cfg.target_update_steps == 0
    K = 8
    due = [it for it in range(101) if target_sync_due(cfg, it, it * K, (it + 1) * K)]
    assert due == [0, 20, 40, 60, 80, 100]
    steps = AQLEngineConfig(target_update_steps=100)
    due = [it for it in range(60) if target_sync_due(steps, it, it * K, (it + 1) * K)]
    assert due == [12, 24, 37, 49]   # learner-step count crosses 100, 200, 300, 400
    off = AQLEngineConfig(target_update_interval=0)
    assert not any(target_sync_due(off, it, 0, 0) for it in range(50))
