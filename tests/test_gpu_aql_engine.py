"""GPU AQL engine (engine/aql.py, aql_engine_kernels.hip) vs the PyTorch reference update.

One fused learner step is compared with the reference AQL_dis learner step
(AQL_dis.py:63-108 + utils.py:44-61) run in fp64 PyTorch on the SAME sampled batch (the
engine's own PER indices / IS weights): Q over the candidates, losses, priorities, every
parameter gradient of both losses (pre-clip) and the parameters after the two clipped Adam
steps.  The vector envs are checked against the envs/classic.py dynamics on the
transitions they inserted into the replay.
"""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _engine(cuda, env_id, fill=2048, **kw):
    from apex_amd.engine.aql import AQLEngine, AQLEngineConfig

    cfg = AQLEngineConfig(env_id=env_id, n_envs=64, capacity=8192, batch_size=32, use_graphs=False, **kw)
    eng = AQLEngine(cfg, cuda)
    with torch.no_grad():  # non-zero biases: every bias path exercised
        g = torch.Generator(device="cpu").manual_seed(3)
        for name, p in eng.model.named_parameters():
            if p.dim() == 1 and "sigma" not in name:
                p.copy_((torch.rand(p.shape, generator=g) * 0.4 - 0.2).to(p.device))
    eng.learner.sync_target()
    eng.publish()
    eng.fill(fill)
    torch.cuda.synchronize()
    return eng


def _ref_models(eng, dt):
    mr = copy.deepcopy(eng.model).to(dt)
    tr = copy.deepcopy(eng.target).to(dt)
    for m in (mr, tr):
        m.proposal.action_var = m.proposal.action_var.to(device=eng.device, dtype=dt)
        m.q.train()
    return mr, tr


def _batch(eng, dt):
    r, L = eng.replay, eng.learner
    idx = L.idx.long()
    s, s2 = r.st[idx].to(dt), r.st2[idx].to(dt)
    a = r.action[idx].long()
    rew, d = r.reward[idx].to(dt), r.done[idx].to(dt)
    am = r.a_mu[idx].to(dt)
    if not eng.cont:
        am = am.reshape(am.shape[0], -1)
    return s, a, rew, s2, d, am, L.w.to(dt)


def _grads(model, names):
    return {n: (p.grad.detach().clone() if p.grad is not None else torch.zeros_like(p))
            for n, p in model.named_parameters() if n in names}


@pytest.mark.parametrize("env_id", ["BipedalWalker-v3", "CartPole-v0", "Pendulum-v0"])
def test_learner_step_matches_reference(cuda, env_id):
    from apex_amd.algo.losses import compute_loss_AQL

    kw = dict(propose_sample=7, uniform_sample=9) if env_id == "Pendulum-v0" else {}
    eng = _engine(cuda, env_id, **kw)
    L, cfg = eng.learner, eng.cfg
    # fp64 reference; the discrete critic casts its candidate input with .float()
    # (model.py candidate encoder), so CartPole runs the reference in fp32
    dt = torch.float64 if eng.cont else torch.float32
    mr, tr = _ref_models(eng, dt)  # snapshot BEFORE the step
    p_before = L.flat.clone()
    L.step()
    torch.cuda.synchronize()
    s, a, rew, s2, d, am, w = _batch(eng, dt)
    B = s.shape[0]

    # --- reference learner step (AQL_dis.compute_td_loss), fp64
    q_values = mr(s, am)
    with torch.no_grad():
        q2_ref = mr.q.candidate_q(s2, am)
        qt2_ref = tr.q.candidate_q(s2, am)
    scale = q_values.detach().abs().max().item() + 1e-6
    assert (L.q_s.double() - q_values.detach()).abs().max().item() <= 1e-4 * scale
    assert (L.q_s2.double() - q2_ref).abs().max().item() <= 1e-4 * scale
    assert (L.qt_s2.double() - qt2_ref).abs().max().item() <= 1e-4 * scale
    dist = mr.proposal.evaluate(mr.q.embedding_feature(s))
    best = am[torch.arange(B, device=am.device), q_values.max(1)[1]].reshape(B, -1)
    loss_p = torch.mean(-dist.log_prob(best) - cfg.ent_lam * dist.entropy())
    opt_p = torch.optim.Adam(mr.proposal.parameters(), cfg.lr)
    opt_p.zero_grad()
    loss_p.backward()
    prop_names = {n for n, _ in mr.named_parameters() if n.startswith("proposal.")}
    g_ref = _grads(mr, prop_names)
    torch.nn.utils.clip_grad_norm_(mr.proposal.parameters(), cfg.max_norm)
    opt_p.step()
    tr.proposal.load_state_dict(mr.proposal.state_dict())
    loss_q, prios = compute_loss_AQL(mr, tr, (s, a, rew, s2, d, am, w), n_steps=cfg.n_steps, gamma=cfg.gamma)
    opt_q = torch.optim.Adam(mr.q.parameters(), cfg.lr)
    opt_q.zero_grad()
    loss_q.backward()
    q_names = {n for n, _ in mr.named_parameters() if n.startswith("q.")}
    g_ref.update(_grads(mr, q_names))
    torch.nn.utils.clip_grad_norm_(mr.q.parameters(), cfg.max_norm)
    opt_q.step()

    # --- losses, priorities
    assert abs(L.loss_q.item() - loss_q.item()) <= 1e-4 * max(1.0, abs(loss_q.item()))
    assert abs(L.loss_p.item() - loss_p.item()) <= 1e-4 * max(1.0, abs(loss_p.item()))
    pr = torch.as_tensor(prios, dtype=torch.float64)
    assert (L.prio.double().cpu() - pr).abs().max().item() <= 1e-4 * pr.abs().max().item()
    # --- gradients (pre-clip), per tensor
    offs = eng.model._flat_offsets  # parameters start at 16-byte offsets of the flat buffer
    for name, p in eng.model.named_parameters():
        n, off = p.numel(), offs[name]
        g = L.grad[off:off + n].double().reshape(p.shape)
        ref = g_ref[name]
        err = (g - ref).norm().item()
        assert err <= 1e-4 * ref.norm().item() + 1e-9, (name, err, ref.norm().item())
    # --- parameters after both clipped Adam steps: |dp| = lr * m/(sqrt(v)+eps) is sign-like on
    # the first step, so compare the update with an lr-relative bound
    sel = torch.cat([torch.arange(offs[n], offs[n] + p.numel()) for n, p in eng.model.named_parameters()])
    sel = sel.to(L.flat.device)
    p_ref = torch.cat([p.detach().reshape(-1) for p in mr.parameters()])
    diff = (L.flat[sel].double() - p_ref).abs()
    moved = (p_ref - p_before[sel].double()).abs()
    assert diff.max().item() <= 2.01 * cfg.lr
    assert (diff > 1e-3 * cfg.lr).float().mean().item() < 1e-3, "more than 0.1% of updates differ"
    assert moved.max().item() > 0.5 * cfg.lr
    # --- proposal hard copy (AQL_dis.py:92) and fresh noise (AQL_dis.py:104-105)
    assert torch.equal(L.tflat[L.P_q:], L.flat[L.P_q:])
    assert L.step_ctr.item() == 1


def test_noise_reset_is_factorised_gaussian(cuda):
    eng = _engine(cuda, "BipedalWalker-v3", fill=512)
    L = eng.learner
    before = L.eps.clone()
    L.step()
    torch.cuda.synchronize()
    a1 = eng.model.q.advantage1
    W = a1.weight_epsilon.double()
    assert not torch.equal(L.eps, before)
    # rank-1: eps_w = f(eps_out) f(eps_in)^T
    sv = torch.linalg.svdvals(W)
    assert sv[1].item() <= 1e-5 * sv[0].item()
    # f(x) = sign(x) sqrt|x| of N(0,1): E f^2 = E|x| = sqrt(2/pi)
    e_all = torch.cat([eng.model.q.advantage1.bias_epsilon, eng.target.q.advantage1.bias_epsilon]).double()
    assert abs((e_all ** 2).mean().item() - np.sqrt(2 / np.pi)) < 0.25
    # online and target draw independent noise
    assert not torch.equal(eng.model.q.advantage1.bias_epsilon, eng.target.q.advantage1.bias_epsilon)


def test_bipedal_env_transitions(cuda):
    eng = _engine(cuda, "BipedalWalker-v3", fill=1024)
    r = eng.replay
    n = len(r)
    s, s2 = r.st[:n].double(), r.st2[:n].double()
    act = r.action[:n].long()
    a_env = r.a_mu[:n][torch.arange(n, device=act.device), act].double().clamp(-1, 1)
    A, Bm, wv = eng.dynA.double(), eng.dynB.double(), eng.dynw.double()
    pred = torch.tanh(s @ A.T + a_env @ Bm.T)
    # s' = tanh(A s + B a + N(0, 0.01)): within ~5 sigma of the noise-free prediction
    assert (s2 - pred).abs().max().item() < 0.06
    rew, done = r.reward[:n].double(), r.done[:n]
    ok = rew > -100
    exp_r = 0.05 * (s2 @ wv) - 0.028 * a_env.abs().sum(1)
    assert (rew[ok] - exp_r[ok]).abs().max().item() < 1e-4
    fell = (s2[:, 0].abs() > 0.995)
    assert torch.equal(fell, rew == -100)
    assert bool((done[fell] == 1).all())


def test_cartpole_env_matches_host_dynamics(cuda):
    from apex_amd import envs

    eng = _engine(cuda, "CartPole-v0", fill=1024)
    r = eng.replay
    n = len(r)
    s, s2 = r.st[:n].cpu().double().numpy(), r.st2[:n].cpu().double().numpy()
    act = r.action[:n].long()
    a_env = r.a_mu[:n, :, 0][torch.arange(n, device=act.device), act].cpu().numpy().astype(int)
    env = envs.make("CartPole-v0").unwrapped
    for i in range(0, n, 7):
        env.reset()
        env.state = tuple(float(x) for x in s[i])
        env.steps_beyond_done = None
        ns, rr, dd, _ = env.step(int(a_env[i]))
        np.testing.assert_allclose(s2[i], ns, rtol=1e-4, atol=1e-5)
        assert rr == r.reward[i].item() == 1.0
        if dd:
            assert r.done[i].item() == 1.0


def test_engine_iterations_graph_replay(cuda):
    """Captured actor + K-learner-step graphs: losses stay finite, the replay fills at E
    transitions per iteration, the learner counter advances K per iteration, episodes end."""
    from apex_amd.engine.aql import AQLEngine, AQLEngineConfig

    cfg = AQLEngineConfig(env_id="CartPole-v0", n_envs=128, capacity=16384, batch_size=32)
    eng = AQLEngine(cfg, cuda)
    eng.fill(1024)
    eng.capture()
    f0 = int(eng.replay.filled.item())
    for _ in range(20):
        eng.iteration()
    torch.cuda.synchronize()
    st = eng.learner.stats()
    assert np.isfinite(st["loss_q"]) and np.isfinite(st["loss_proposal"])
    assert st["steps"] == 20 * eng.K
    assert int(eng.replay.filled.item()) == f0 + 20 * cfg.n_envs
    eps = eng.finished_episodes()
    assert len(eps) > 0 and all(1 <= ln <= 200 for _, ln in eps)
    # actors hold the published online weights
    assert torch.equal(eng.actor_flat, eng.learner.flat)


@pytest.mark.parametrize("env_id", ["BipedalWalker-v3", "CartPole-v0"])
def test_acting_q_mfma_matches_fp64(cuda, env_id):
    """Acting Q on the learner's MFMA candidate forward (aql_act_q, the engine default) and the
    one-wave-per-item kernel (aql_candidate_q) against the fp64 reference Q_Network over the
    engine's own candidate sets."""
    eng = _engine(cuda, env_id, fill=256)
    h, s = eng.hip, torch.cuda.current_stream().cuda_stream
    E, T = eng.E, eng.T
    h.aql_propose(eng.actor_net, eng.obs_buf.data_ptr(), E, eng.low.data_ptr(), eng.high.data_ptr(),
                  eng.var.data_ptr(), 77, eng.actor_ctr.data_ptr(), eng.amu.data_ptr(), 0, s)
    h.aql_noisy_eff(eng.actor_net, eng.ws.data_ptr(), s)
    h.aql_act_q(eng.actL, s)
    torch.cuda.synchronize()
    q_mfma = eng.qbuf.clone()
    h.aql_candidate_q(eng.actor_net, eng.ws.data_ptr(), eng.obs_buf.data_ptr(), eng.amu.data_ptr(), E,
                      eng.qbuf.data_ptr(), s)
    torch.cuda.synchronize()
    q_scalar = eng.qbuf.clone()
    ref = copy.deepcopy(eng.actor_model).double()
    with torch.no_grad():  # Q_Network.candidate_q in fp64 (its discrete branch casts to fp32)
        qn = ref.q
        a_out = qn.action_out(eng.amu.double().reshape(E * T, eng.adim)).reshape(E, T, qn.A_OUT)
        q_f = qn.q_feature(eng.obs_buf.double()).repeat(1, T).reshape(E, T, qn.F_OUT)
        q64 = qn.forward(torch.relu(torch.cat([a_out, q_f], dim=2))).reshape(E, T)
    for q in (q_mfma, q_scalar):
        err = float((q.double() - q64).abs().max() / q64.abs().max().clamp_min(1e-30))
        assert err < 1e-5, err


def test_overlapped_acting_graphs_equal_eager(cuda):
    """Overlap mode (acting on its own stream, transitions staged and applied by the learner's
    graph): captured graphs == the same schedule run eagerly on one stream, bit for bit, and
    the ring advances E transitions per iteration."""
    from apex_amd.engine.aql import AQLEngine, AQLEngineConfig

    def run(graphs: bool):
        cfg = AQLEngineConfig(env_id="CartPole-v0", n_envs=128, capacity=16384, batch_size=32, overlap=True, seed=5)
        eng = AQLEngine(cfg, cuda)
        eng.fill(1024)
        if graphs:
            eng.capture()
        f0 = int(eng.replay.filled.item())
        for _ in range(12):
            eng.iteration()
        torch.cuda.synchronize()
        assert int(eng.replay.filled.item()) == f0 + 12 * cfg.n_envs
        assert eng.learner.stats()["steps"] == 12 * eng.K
        return eng.learner.flat.clone(), eng.replay.leaf_sum.clone(), eng.obs_buf.clone()

    a, b = run(False), run(True)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_fused_sequence_equals_reference_sequence(cuda):
    """The engine's four-launch step (the forward draws its own PER rows or uses the rows the
    previous step's update launch drew; the priority write as extra workgroups of the backward
    and gradient launches; both Adam steps + noise reset + proposal copy + next draw in one
    update launch) == the reference sequence of separate launches (per_sample, forward,
    backward, per_write_batch, gradients, adam_step2, noise reset): same rows, IS weights,
    tree, loss, parameters, moments, noise and target after several iterations, eager and
    graph-captured, bit for bit."""
    from apex_amd.engine.aql import AQLEngine, AQLEngineConfig

    out = []
    for fused in (False, True):
        cfg = AQLEngineConfig(env_id="BipedalWalker-v3", n_envs=64, capacity=8192, batch_size=32, seed=9, fused=fused)
        eng = AQLEngine(cfg, cuda)
        L = eng.learner
        assert L.fused == fused and L.predraw == fused and (L.U is not None) == fused
        eng.fill(1024)
        for _ in range(5):
            eng.iteration()
        eng.capture()  # and graph-captured
        for _ in range(3):
            eng.iteration()
        torch.cuda.synchronize()
        r = eng.replay
        out.append((L.idx.clone(), L.w.clone(), L.flat.clone(), L.m.clone(), L.v.clone(), L.eps.clone(),
                    L.teps.clone(), L.tflat.clone(), L.eff_on.clone(), L.eff_tg.clone(), L.loss_q.clone(),
                    L.loss_p.clone(), L.prio.clone(), L.norms_q.clone(), L.norms_p.clone(), L.step_ctr.clone(),
                    r.leaf_sum.clone(), r.node_sum[-1].clone(), r.max_prio.clone()))
    names = ("idx", "w", "flat", "m", "v", "eps", "teps", "tflat", "eff_on", "eff_tg", "loss_q", "loss_p", "prio",
             "norms_q", "norms_p", "step", "leaf_sum", "root", "max_prio")
    for name, x, y in zip(names, out[0], out[1]):
        assert torch.equal(x, y), (name, (x.double() - y.double()).abs().max().item())


def test_step_gate_runs_only_the_paid_steps(cuda):
    """The device step gate (the central learner's rows-applied replay ratio): K = 4 captured
    steps with gate = 2 train exactly like K = 2 ungated steps -- the gated-off steps' launches
    change nothing (parameters, moments, tree, step counter), eager and graph-captured."""
    from apex_amd.engine.aql import AQLEngine, AQLEngineConfig

    def run(K, n):
        cfg = AQLEngineConfig(env_id="CartPole-v0", n_envs=64, capacity=8192, batch_size=32, seed=3, learner_steps=K)
        eng = AQLEngine(cfg, cuda)
        eng.fill(1024)
        gate = None if n is None else torch.full((1,), n, dtype=torch.int32, device=cuda)
        for _ in range(3):
            eng.actor_step()
            eng.learn_steps(gate=gate)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            eng.learn_steps(gate=gate)
        for _ in range(2):
            eng.actor_step()
            g.replay()
        torch.cuda.synchronize()
        L = eng.learner
        return (L.flat.clone(), L.m.clone(), L.v.clone(), L.eps.clone(), eng.replay.leaf_sum.clone(),
                L.step_ctr.clone())

    a, b = run(4, 2), run(2, None)
    assert int(a[-1].item()) == 5 * 2
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_forward_tile_groups_bit_identical(cuda):
    """The learner forward's work split (candidate tiles per workgroup: one, a few, all of a
    sample's) changes only which waves compute a tile: same Q rows, same training."""
    from apex_amd.engine.aql import AQLEngine, AQLEngineConfig

    out = []
    for groups in (0, 1, 3, 13, 4):
        cfg = AQLEngineConfig(env_id="BipedalWalker-v3", n_envs=64, capacity=8192, batch_size=32, seed=5,
                              fwd_tile_groups=groups)
        eng = AQLEngine(cfg, cuda)
        eng.fill(1024)
        for _ in range(4):
            eng.iteration()
        torch.cuda.synchronize()
        L = eng.learner
        out.append((L.q_s.clone(), L.q_s2.clone(), L.qt_s2.clone(), L.idx.clone(), L.flat.clone()))
    for k in range(1, len(out)):
        for name, x, y in zip(("q_s", "q_s2", "qt_s2", "idx", "flat"), out[0], out[k]):
            assert torch.equal(x, y), (k, name)


@pytest.mark.parametrize("env_id", ["BipedalWalker-v3", "CartPole-v0"])
def test_propose_mu_matches_fp64_and_fused_eff(cuda, env_id):
    """aql_propose (four states per workgroup, dist_feature.0 staged in LDS): the proposal mean
    against the fp64 reference Proposal_Network, and the effective-weight workgroups riding in
    the same launch == aql_noisy_eff, with the candidate sets unchanged by them."""
    eng = _engine(cuda, env_id, fill=256)
    h, s = eng.hip, torch.cuda.current_stream().cuda_stream
    E = eng.E
    ref = copy.deepcopy(eng.actor_model).double()
    with torch.no_grad():
        mu64 = ref.proposal.dist_feature(ref.q.embedding_feature(eng.obs_buf.double()))
    A = mu64.shape[1]
    mu = torch.zeros(E, A, device=cuda)
    h.aql_propose(eng.actor_net, eng.obs_buf.data_ptr(), E, eng.low.data_ptr(), eng.high.data_ptr(),
                  eng.var.data_ptr(), 77, eng.actor_ctr.data_ptr(), eng.amu.data_ptr(), mu.data_ptr(), s)
    h.aql_noisy_eff(eng.actor_net, eng.ws.data_ptr(), s)
    torch.cuda.synchronize()
    am0, ws0 = eng.amu.clone(), eng.ws.clone()
    err = float((mu.double() - mu64).abs().max() / mu64.abs().max().clamp_min(1e-30))
    assert err < 1e-5, err
    eng.ws.zero_()
    h.aql_propose(eng.actor_net, eng.obs_buf.data_ptr(), E, eng.low.data_ptr(), eng.high.data_ptr(),
                  eng.var.data_ptr(), 77, eng.actor_ctr.data_ptr(), eng.amu.data_ptr(), 0, s, eng.ws.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(eng.amu, am0)
    assert torch.equal(eng.ws, ws0)


def test_last_step_publishes_acting_copies(cuda):
    """Serial engine: the iteration's last SGD step writes the acting weights and online noise
    from its update launch (no publish copies) -- they equal the learner's after every
    iteration, eager and graph-replayed."""
    from apex_amd.engine.aql import AQLEngine, AQLEngineConfig

    eng = AQLEngine(AQLEngineConfig(env_id="BipedalWalker-v3", n_envs=64, capacity=8192, batch_size=32, seed=4), cuda)
    L = eng.learner
    assert L.U_pub is not None
    eng.fill(1024)
    for it in range(6):
        if it == 3:
            eng.capture()
        eng.iteration()
        torch.cuda.synchronize()
        assert torch.equal(eng.actor_flat, L.flat), it
        assert torch.equal(eng.actor_eps, L.eps), it


@pytest.mark.parametrize("env_id", ["BipedalWalker-v3", "CartPole-v0"])
def test_fused_acting_tail_equals_separate_launches(cuda, env_id):
    """The serial engine's one-launch acting tail (aql_act_tail: eps-greedy select + env step +
    ring tree write + counter bumps + the learner's PER beta from a device iteration counter)
    == select, env step, per_write_leaves and the host's beta fill as separate launches: same
    replay rows, tree, counters, env state, beta and learner after fill + eager and
    graph-captured iterations, bit for bit."""
    from apex_amd.engine.aql import AQLEngine, AQLEngineConfig

    out = []
    for fused in (False, True):
        cfg = AQLEngineConfig(env_id=env_id, n_envs=96, capacity=8192, batch_size=32, seed=13, fused_acting=fused,
                              max_step=40)  # (a short beta horizon: beta moves every iteration)
        eng = AQLEngine(cfg, cuda)
        assert (eng._tail is not None) == fused
        eng.fill(1024)
        for _ in range(4):
            eng.iteration()
        eng.capture()
        for _ in range(3):
            eng.iteration()
        torch.cuda.synchronize()
        r, L = eng.replay, eng.learner
        out.append((r.st.clone(), r.st2.clone(), r.action.clone(), r.reward.clone(), r.done.clone(), r.a_mu.clone(),
                    r.leaf_sum.clone(), r.node_sum[0].clone(), r.node_sum[-1].clone(), r.filled.clone(),
                    eng.actor_ctr.clone(), eng.obs_buf.clone(), eng.ep_len.clone(), eng.ep_ret.clone(),
                    eng.ep_count.clone(), L.beta.clone(), L.idx.clone(), L.flat.clone()))
    names = ("st", "st2", "action", "reward", "done", "a_mu", "leaf_sum", "level1", "root", "filled", "actor_ctr",
             "obs", "ep_len", "ep_ret", "ep_count", "beta", "idx", "flat")
    for name, x, y in zip(names, out[0], out[1]):
        assert torch.equal(x, y), (name, (x.double() - y.double()).abs().max().item())
    assert out[1][15].item() != AQLEngineConfig().beta_start  # the device beta moved
