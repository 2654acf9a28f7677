"""Fused learner backward pieces vs the separate reference kernels / torch fp32:
dqn_heads_bwd (loss + heads backward + head-gradient partials), the priority mix in the
tree write, and grad_finalize (one launch for all batch-sliced reductions)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(dev, B=512, A=18, C=4096, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    q = torch.randn(B, A, device=dev, generator=g)
    q2 = torch.randn(B, A, device=dev, generator=g)
    q2[:, 3] = q2[:, 5]  # ties in the argmax
    q2t = torch.randn(B, A, device=dev, generator=g)
    act = torch.randint(0, A, (C,), device=dev, generator=g, dtype=torch.int32)
    rew = torch.randn(C, device=dev, generator=g)
    done = (torch.rand(C, device=dev, generator=g) < 0.2).float()
    idx = torch.randint(0, C, (B,), device=dev, generator=g, dtype=torch.int32)
    w = torch.rand(B, device=dev, generator=g) + 0.2
    h = torch.relu(torch.randn(B, 256, device=dev, generator=g))
    wa = torch.randn(A, 128, device=dev, generator=g) * 0.1
    wv = torch.randn(1, 128, device=dev, generator=g) * 0.1
    return q, q2, q2t, act, rew, done, idx, w, h, wa, wv


@pytest.mark.parametrize("B", [512, 37])
def test_dqn_heads_bwd_matches_separate_kernels(cuda, B):
    from apex_amd import ops

    hip = ops.hip()
    A, gn = 18, 0.99 ** 3
    q, q2, q2t, act, rew, done, idx, w, h, wa, wv = _setup(cuda, B, A)
    s = torch.cuda.current_stream().cuda_stream
    # reference: dqn_loss + heads_bwd + heads_wgrad
    loss = torch.zeros(1, device=cuda)
    dq = torch.zeros(B, A, device=cuda)
    prio = torch.zeros(B, device=cuda)
    hip.dqn_loss(q.data_ptr(), q2.data_ptr(), q2t.data_ptr(), A, act.data_ptr(), rew.data_ptr(), done.data_ptr(),
                 idx.data_ptr(), w.data_ptr(), B, A, gn, loss.data_ptr(), dq.data_ptr(), prio.data_ptr(), s)
    dA = torch.zeros(B, A + 1, device=cuda)
    dz = torch.zeros(B, 256, device=cuda)
    dz_bf = torch.zeros(B, 256, dtype=torch.bfloat16, device=cuda)
    hip.heads_bwd(dq.data_ptr(), h.data_ptr(), wa.data_ptr(), wv.data_ptr(), dA.data_ptr(), dz.data_ptr(),
                  dz_bf.data_ptr(), B, A, s)
    ref = {k: torch.zeros(n, device=cuda) for k, n in
           (("wa", A * 128), ("ba", A), ("wv", 128), ("bv", 1), ("ba1", 128), ("bv1", 128))}
    hws = torch.zeros(hip.heads_wgrad_workspace_floats(A), device=cuda)
    hip.heads_wgrad(dA.data_ptr(), h.data_ptr(), dz.data_ptr(), B, A, hws.data_ptr(), ref["wa"].data_ptr(),
                    ref["ba"].data_ptr(), ref["wv"].data_ptr(), ref["bv"].data_ptr(), ref["ba1"].data_ptr(),
                    ref["bv1"].data_ptr(), s)
    # fused
    blocks = hip.dqn_heads_bwd_blocks(B)
    part = torch.zeros(blocks * ((A + 1) * 128 + (A + 1) + 256), device=cuda)
    delta = torch.zeros(B, device=cuda)
    lw = torch.zeros(B, device=cuda)
    dz2 = torch.zeros(B, 256, dtype=torch.bfloat16, device=cuda)
    step = torch.full((1,), 41, dtype=torch.int64, device=cuda)
    snap = torch.zeros(1, dtype=torch.int64, device=cuda)
    hip.dqn_heads_bwd({"q": q.data_ptr(), "q2": q2.data_ptr(), "q2t": q2t.data_ptr(), "act": act.data_ptr(),
                       "rew": rew.data_ptr(), "done": done.data_ptr(), "idx": idx.data_ptr(), "w": w.data_ptr(),
                       "h": h.data_ptr(), "w_adv2": wa.data_ptr(), "w_val2": wv.data_ptr(), "delta": delta.data_ptr(),
                       "lw": lw.data_ptr(), "dz_bf": dz2.data_ptr(), "part": part.data_ptr(),
                       "step": step.data_ptr(), "step_snap": snap.data_ptr()}, B, A, gn, s)
    got = {k: torch.zeros_like(v) for k, v in ref.items()}
    job = hip.heads_finalize_job(blocks, A, part.data_ptr(), got["wa"].data_ptr(), got["ba"].data_ptr(),
                                 got["wv"].data_ptr(), got["bv"].data_ptr(), got["ba1"].data_ptr(),
                                 got["bv1"].data_ptr())
    hip.grad_finalize([job], s)
    torch.cuda.synchronize()
    assert int(snap.item()) == 41
    # TD errors -> the same mixed priorities and loss
    dmax = delta.max()
    torch.testing.assert_close(0.9 * dmax + 0.1 * delta + 1e-6, prio, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(lw.sum() / B, loss[0], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(dz2.float(), dz_bf.float(), rtol=2e-2, atol=1e-6)
    for k in ref:
        torch.testing.assert_close(got[k], ref[k], rtol=1e-4, atol=1e-6, msg=k)


def test_tree_write_priority_mix(cuda):
    """PrioMix in the sorted tree write == dqn_loss priorities written directly."""
    from apex_amd.engine.hbm_replay import HBMReplay

    B, C = 512, 8192
    g = torch.Generator(device=cuda).manual_seed(3)
    rp1 = HBMReplay(C, 64, 3, 0.6, cuda)
    rp2 = HBMReplay(C, 64, 3, 0.6, cuda)
    idx = torch.randint(0, C, (B,), device=cuda, generator=g, dtype=torch.int32)  # duplicates included
    delta = torch.rand(B, device=cuda, generator=g) * 3
    lw = torch.rand(B, device=cuda, generator=g)
    prio = 0.9 * delta.max() + 0.1 * delta + 1e-6
    out_p = torch.zeros(B, device=cuda)
    loss = torch.zeros(1, device=cuda)
    rp2.write_priorities(idx, None, dedup=True, mix=(delta, lw, out_p, loss))
    rp1.write_priorities(idx, out_p.clone(), dedup=True)  # the mixed values, written directly
    torch.cuda.synchronize()
    assert torch.equal(rp1.leaf_sum, rp2.leaf_sum)
    for a, b in zip(rp1.node_sum, rp2.node_sum):
        assert torch.equal(a, b)
    assert torch.equal(rp1.max_prio, rp2.max_prio)
    assert math.isclose(loss.item(), lw.sum().item() / B, rel_tol=1e-5)
    torch.testing.assert_close(out_p, prio, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("C,B,E", [(4096, 512, 256), (8192, 512, 256), (1 << 21, 512, 256), (8192, 32, 16),
                                   (1 << 21, 64, 32)])
def test_batched_tree_write_equals_sequential_writes(cuda, C, B, E):
    """write_batch (actor rows + mixed learner priorities, dedup by claims, wide level
    kernels + last-block top levels -- or, at <= 64 rows, every level inside the leaves
    workgroup) leaves the tree bit-identical to the old sequential path (ring write, then the
    sorted dedup write), repeatedly (claims released)."""
    from apex_amd.engine.hbm_replay import HBMReplay

    g = torch.Generator(device=cuda).manual_seed(11)
    rp1 = HBMReplay(C, E, 3, 0.6, cuda)
    rp2 = HBMReplay(C, E, 3, 0.6, cuda)
    c1, c2 = torch.zeros(1, dtype=torch.int64, device=cuda), torch.zeros(1, dtype=torch.int64, device=cuda)
    for it in range(4):
        base = (it * E) % C
        slots = (torch.arange(E, device=cuda, dtype=torch.int32) + base) % C
        aprio = torch.rand(E, device=cuda, generator=g) * 2 + 0.05
        idx = torch.randint(0, C, (B,), device=cuda, generator=g, dtype=torch.int32)
        idx[:E // 4] = slots[:E // 4]            # learner samples that the actor rows just wrote
        idx[E // 4:E // 2] = idx[:E // 4]        # and duplicates
        delta = torch.rand(B, device=cuda, generator=g) * 3
        lw = torch.rand(B, device=cuda, generator=g)
        p1, p2 = torch.zeros(B, device=cuda), torch.zeros(B, device=cuda)
        l1, l2 = torch.zeros(1, device=cuda), torch.zeros(1, device=cuda)
        rp1.write_priorities(slots, aprio, dedup=False, bumps=((rp1.filled, E),))
        rp1.write_priorities(idx, None, dedup=True, bumps=((c1, 1),), mix=(delta, lw, p1, l1))
        rp2.write_batch(pre=(slots, aprio, rp2.filled), idx=idx, bump=c2, mix=(delta, lw, p2, l2))
        torch.cuda.synchronize()
        assert torch.equal(rp1.leaf_sum, rp2.leaf_sum) and torch.equal(rp1.leaf_min, rp2.leaf_min), it
        for a, b in zip(rp1.node_sum + rp1.node_min, rp2.node_sum + rp2.node_min):
            assert torch.equal(a, b), it
        assert torch.equal(rp1.max_prio, rp2.max_prio) and torch.equal(rp1.filled, rp2.filled)
        assert torch.equal(c1, c2) and torch.equal(p1, p2) and torch.equal(l1, l2)
    assert int((rp2.owner != -1).sum()) == 0 and int(rp2.ticket.item()) == 0
    # the root equals a full recomputation from the leaves
    full = rp2.leaf_sum.double().sum()
    torch.testing.assert_close(rp2.node_sum[-1][0], full, rtol=1e-12, atol=0)
    assert rp2.node_min[-1][0].item() == rp2.leaf_min.min().item()
