"""Fused learner kernels vs plain PyTorch fp32 references."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _loss_inputs(B, A, dev, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    q = (torch.randn(B, A, generator=g) * 3).to(dev)
    q2 = torch.randn(B, A, generator=g).to(dev)
    q2t = torch.randn(B, A, generator=g).to(dev)
    a = torch.randint(0, A, (B,), generator=g).to(dev).int()
    r = torch.randn(B, generator=g).to(dev)
    d = (torch.rand(B, generator=g) < 0.2).float().to(dev)
    w = torch.rand(B, generator=g).to(dev) + 0.1
    return q, q2, q2t, a, r, d, w


@pytest.mark.parametrize("B,A", [(512, 18), (64, 6), (1000, 3)])
def test_dqn_loss_matches_torch(cuda, B, A):
    from apex_amd import ops
    from apex_amd.algo.losses import huber_weighted

    hip = ops.hip()
    q, q2, q2t, a, r, d, w = _loss_inputs(B, A, cuda)
    gn = 0.99 ** 3
    loss = torch.empty(1, device=cuda)
    dq = torch.empty(B, A, device=cuda)
    prio = torch.empty(B, device=cuda)
    s = torch.cuda.current_stream().cuda_stream
    hip.dqn_loss(q.data_ptr(), q2.data_ptr(), q2t.data_ptr(), A, a.data_ptr(), r.data_ptr(), d.data_ptr(), 0,
                 w.data_ptr(), B, A, gn, loss.data_ptr(), dq.data_ptr(), prio.data_ptr(), s)
    qr = q.clone().requires_grad_(True)
    q_a = qr.gather(1, a.long().unsqueeze(1)).squeeze(1)
    a_star = q2.max(1)[1].unsqueeze(1)
    y = r + gn * q2t.gather(1, a_star).squeeze(1) * (1 - d)
    td = torch.abs(y.detach() - q_a)
    ref_loss = huber_weighted(td, w)
    ref_loss.backward()
    ref_prio = 0.9 * td.max() + 0.1 * td + 1e-6
    torch.testing.assert_close(loss[0], ref_loss.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(prio, ref_prio.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dq, qr.grad, rtol=1e-5, atol=1e-8)


def _seg_handle(hip, shapes):
    return None, int(sum(int(np.prod(sh)) for sh in shapes))


@pytest.mark.parametrize("centered", [True, False])
@pytest.mark.parametrize("size", ["full", "small"])
def test_rmsprop_clip_matches_torch(cuda, centered, size):
    """``small`` (~43k parameters) runs the optimizer's one-pass path (one element per thread,
    every load in flight before the norm reduce), ``full`` (~445k) its grid-stride loop."""
    from apex_amd import ops

    hip = ops.hip()
    shapes = [(32, 4, 8, 8), (32,), (64, 32, 4, 4), (64,), (128, 3136), (128,), (18, 128), (18,)]
    if size == "small":
        shapes = [sh for sh in shapes if sh != (128, 3136)]
    seg, P = _seg_handle(hip, shapes)
    g = torch.Generator(device="cpu").manual_seed(3)
    params = [torch.randn(*sh, generator=g).to(cuda) for sh in shapes]
    flat = torch.cat([p.reshape(-1) for p in params]).contiguous()
    sq = torch.zeros(P, device=cuda)
    ga = torch.zeros(P, device=cuda)
    ref = [p.clone().requires_grad_(True) for p in params]
    opt = torch.optim.RMSprop(ref, lr=6.25e-5, alpha=0.95, eps=1.5e-7, centered=centered)
    hp = hip.RMSpropParams(6.25e-5, 0.95, 1.5e-7, 40.0, 1.0, 0, 0, centered)
    partials = torch.zeros(hip.grad_norm_partials(), dtype=torch.float64, device=cuda)
    norms = torch.zeros(4, device=cuda)
    step = torch.zeros(1, dtype=torch.int64, device=cuda)
    s = torch.cuda.current_stream().cuda_stream
    for it in range(5):
        grads = [torch.randn(*sh, generator=g).to(cuda) * (20 if it % 2 else 0.01) for sh in shapes]
        gflat = torch.cat([x.reshape(-1) for x in grads]).contiguous()
        hip.grad_sumsq(gflat.data_ptr(), P, partials.data_ptr(), s)
        hip.rmsprop_step(flat.data_ptr(), gflat.data_ptr(), sq.data_ptr(), ga.data_ptr(), P, partials.data_ptr(),
                         partials.numel(), hp, step.data_ptr(), norms.data_ptr(), s)
        for p, gr in zip(ref, grads):
            p.grad = gr.clone()
        l2 = torch.nn.utils.clip_grad_norm_(ref, 40.0)
        refnorm = sum(gr.norm(2) ** 0.5 for gr in grads) ** 0.5
        opt.step()
        torch.testing.assert_close(norms[0], l2, rtol=1e-5, atol=1e-5)
        assert refnorm > 0
    torch.testing.assert_close(flat, torch.cat([p.detach().reshape(-1) for p in ref]), rtol=1e-5, atol=1e-6)


def test_adam_matches_torch(cuda):
    from apex_amd import ops

    hip = ops.hip()
    shapes = [(64, 16), (64,), (3, 64)]
    seg, P = _seg_handle(hip, shapes)
    g = torch.Generator(device="cpu").manual_seed(5)
    params = [torch.randn(*sh, generator=g).to(cuda) for sh in shapes]
    flat = torch.cat([p.reshape(-1) for p in params]).contiguous()
    m = torch.zeros(P, device=cuda)
    v = torch.zeros(P, device=cuda)
    ref = [p.clone().requires_grad_(True) for p in params]
    opt = torch.optim.Adam(ref, lr=1e-3)
    hp = hip.AdamParams(1e-3, max_norm=0.0)
    partials = torch.zeros(hip.grad_norm_partials(), dtype=torch.float64, device=cuda)
    step = torch.zeros(1, dtype=torch.int64, device=cuda)
    s = torch.cuda.current_stream().cuda_stream
    for it in range(6):
        grads = [torch.randn(*sh, generator=g).to(cuda) for sh in shapes]
        gflat = torch.cat([x.reshape(-1) for x in grads]).contiguous()
        hip.grad_sumsq(gflat.data_ptr(), P, partials.data_ptr(), s)
        hip.adam_step(flat.data_ptr(), gflat.data_ptr(), m.data_ptr(), v.data_ptr(), P, partials.data_ptr(),
                      partials.numel(), hp, step.data_ptr(), 0, s)
        hip.bump_counter(step.data_ptr(), 1, 1, s)
        for p, gr in zip(ref, grads):
            p.grad = gr.clone()
        opt.step()
    torch.testing.assert_close(flat, torch.cat([p.detach().reshape(-1) for p in ref]), rtol=1e-5, atol=1e-6)


def test_learner_step_end_to_end(cuda):
    """Engine slice: fill replay from GPU actors, learner steps (eager and graphed)."""
    from apex_amd.engine.apex import ApexEngine, EngineConfig
    from apex_amd.engine.learner import LearnerConfig

    cfg = EngineConfig(n_envs=64, replay_capacity=16384, threshold_size=2048, learner=LearnerConfig(batch_size=128))
    eng = ApexEngine(cfg, cuda)
    eng.fill()
    before = eng.learner.flat.clone()
    for _ in range(3):
        eng.train_step()
    torch.cuda.synchronize()
    st = eng.learner.stats()
    assert np.isfinite(st["loss"]) and st["grad_norm_l2"] > 0
    assert not torch.equal(before, eng.learner.flat)
    # grads landed in the flat buffer (parameters' .grad are views of it)
    assert eng.learner.flat_grad.abs().sum() > 0
    eng.capture()
    for _ in range(5):
        eng.train_step()
    torch.cuda.synchronize()
    st2 = eng.learner.stats()
    assert np.isfinite(st2["loss"])
    assert int(eng.learner.step_counter.item()) == 3 + 3 + 5  # eager + capture warmup + graphed
    sd = eng.learner.model.state_dict()
    assert list(sd)[:2] == ["features.0.weight", "features.0.bias"]
    assert sd["advantage.0.weight"].shape == (128, 3136) and sd["advantage.2.weight"].shape == (18, 128)


def test_optimizer_refuses_packed_copies_without_maps(cuda):
    """Packed copies (an arena) need both scatter maps: the launch is refused on the host
    instead of dereferencing a null map on the device."""
    from apex_amd import ops

    hip = ops.hip()
    P = 1024
    x = [torch.zeros(P, device=cuda) for _ in range(4)]
    partials = torch.zeros(hip.grad_norm_partials(), dtype=torch.float64, device=cuda)
    norms = torch.zeros(4, device=cuda)
    step = torch.zeros(1, dtype=torch.int64, device=cuda)
    arena = torch.zeros(P, device=cuda)
    hp = hip.RMSpropParams(6.25e-5, 0.95, 1.5e-7, 40.0, 1.0, 0, 0, True)
    with pytest.raises(ValueError, match="scatter maps"):
        hip.rmsprop_step(x[0].data_ptr(), x[1].data_ptr(), x[2].data_ptr(), x[3].data_ptr(), P, partials.data_ptr(),
                         partials.numel(), hp, step.data_ptr(), norms.data_ptr(), torch.cuda.current_stream().cuda_stream,
                         arena_f32=arena.data_ptr())

