"""HBM replay kernels vs host references (fp64 numpy oracles)."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _tree_oracle(leaf_sum, sizes):
    levels = [np.asarray(leaf_sum, dtype=np.float64)]
    for n in sizes[1:]:
        prev = levels[-1]
        pad = np.zeros(n * 64)
        pad[:len(prev)] = prev
        levels.append(pad.reshape(n, 64).sum(1))
    return levels


def test_tree_write_update_dedup(cuda):
    from apex_amd.engine.hbm_replay import HBMReplay

    C = 5000
    rp = HBMReplay(C, n_envs=16, device=cuda, alpha=0.6)
    rng = np.random.RandomState(0)
    host = np.zeros(C)
    hmin = np.full(C, np.inf)
    for _ in range(5):
        idx = rng.randint(0, C, size=700).astype(np.int32)
        pr = rng.uniform(0.01, 3.0, size=700).astype(np.float32)
        for i, p in zip(idx, pr):  # sequential => last write wins
            host[i] = float(np.float32(p) ** np.float32(0.6))
            hmin[i] = host[i]
        rp.write_priorities(torch.from_numpy(idx).to(cuda), torch.from_numpy(pr).to(cuda), dedup=True)
    torch.cuda.synchronize()
    leaf = rp.leaf_sum.cpu().numpy()
    np.testing.assert_allclose(leaf, host, rtol=2e-6, atol=1e-7)
    levels = _tree_oracle(leaf, rp.level_sizes)
    for k, t in enumerate(rp.node_sum):
        np.testing.assert_allclose(t.cpu().numpy(), levels[k + 1], rtol=1e-12, atol=1e-9)
    assert rp.min_priority() == pytest.approx(np.min(leaf[leaf > 0]), rel=1e-6)
    assert rp.total_priority() == pytest.approx(leaf.astype(np.float64).sum(), rel=1e-12)


def test_tree_ring_writes_fused(cuda):
    """Actor-style unique ring-ordered chunks (incl. the wrap) take the single-launch path
    (leaves + every level in one workgroup); tree must equal the fp64 oracle."""
    from apex_amd.engine.hbm_replay import HBMReplay

    C, E = 70000, 256
    rp = HBMReplay(C, n_envs=E, device=cuda, alpha=1.0)
    rng = np.random.RandomState(3)
    host = np.zeros(C)
    start = C - 3 * E + 17  # the 4th chunk wraps around the ring end
    for k in range(9):
        idx = ((start + k * E + np.arange(E)) % C).astype(np.int32)
        pr = rng.uniform(0.0, 2.0, size=E).astype(np.float32)
        pr[::11] = 0.0  # "no transition emitted": zero mass
        host[idx] = pr
        rp.write_priorities(torch.from_numpy(idx).to(cuda), torch.from_numpy(pr).to(cuda), dedup=False)
    torch.cuda.synchronize()
    leaf = rp.leaf_sum.cpu().numpy()
    np.testing.assert_allclose(leaf, host, rtol=1e-6, atol=0)
    levels = _tree_oracle(leaf, rp.level_sizes)
    for k, t in enumerate(rp.node_sum):
        np.testing.assert_allclose(t.cpu().numpy(), levels[k + 1], rtol=1e-12, atol=1e-9)
    assert rp.min_priority() == pytest.approx(np.min(leaf[leaf > 0]), rel=1e-6)


@pytest.mark.parametrize("E,R", [(448, 7), (1024, 3), (2048, 2)])
def test_tree_ring_writes_fused_multi_region(cuda, E, R):
    """The central learner's ingest write: R links' ring-ordered rows (each link's slots
    contiguous in its own region, missing packets as -1 holes) as ONE fused launch of up to
    4096 slots (leaves + every level in one workgroup); tree must equal the fp64 oracle."""
    from apex_amd.engine.hbm_replay import HBMReplay

    C = 2_000_000
    rp = HBMReplay(C, n_envs=E, device=cuda, alpha=0.6)
    rng = np.random.RandomState(E + R)
    host = np.zeros(C)
    C_r = C // R
    for step in range(3):
        parts = []
        for r in range(R):
            base = r * C_r + (step * E + 5 * r) % (C_r - E)
            idx = (base + np.arange(E)).astype(np.int32)
            if (r + step) % 4 == 3:  # a link with nothing ready this step
                idx[:] = -1
            parts.append(idx)
        idx = np.concatenate(parts)
        pr = rng.uniform(0.01, 2.0, size=idx.size).astype(np.float32)
        ok = idx >= 0
        host[idx[ok]] = pr[ok].astype(np.float64) ** 0.6
        rp.write_priorities(torch.from_numpy(idx).to(cuda), torch.from_numpy(pr).to(cuda), dedup=False)
    torch.cuda.synchronize()
    leaf = rp.leaf_sum.cpu().numpy()
    np.testing.assert_allclose(leaf, host, rtol=2e-6, atol=0)
    levels = _tree_oracle(leaf, rp.level_sizes)
    for k, t in enumerate(rp.node_sum):
        np.testing.assert_allclose(t.cpu().numpy(), levels[k + 1], rtol=1e-12, atol=1e-9)


def test_sample_stratified_and_weights(cuda):
    from apex_amd.engine.hbm_replay import HBMReplay

    C = 3000
    rp = HBMReplay(C, n_envs=8, device=cuda, alpha=1.0)
    rng = np.random.RandomState(1)
    pr = rng.uniform(0.1, 5.0, size=C).astype(np.float32)
    pr[::7] = 0.0  # empty slots: no mass
    idx = torch.arange(C, dtype=torch.int32, device=cuda)
    rp.write_priorities(idx, torch.from_numpy(pr).to(cuda), dedup=False)
    rp.filled.fill_(C)
    B = 256
    out_i = torch.empty(B, dtype=torch.int32, device=cuda)
    out_w = torch.empty(B, dtype=torch.float32, device=cuda)
    counts = np.zeros(C)
    leaf = rp.leaf_sum.cpu().numpy().astype(np.float64)
    cum = np.cumsum(leaf)
    total = cum[-1]
    pmin = leaf[leaf > 0].min()
    for c in range(200):
        ctr = torch.tensor([c], dtype=torch.int64, device=cuda)
        rp.sample_indices(B, out_i, out_w, ctr, beta=0.4)
        ii = out_i.cpu().numpy()
        ww = out_w.cpu().numpy()
        assert (leaf[ii] > 0).all(), "sampled an empty slot"
        # stratification: sample i falls in stratum i of the cumulative mass
        lo = np.where(ii > 0, cum[ii - 1], 0.0)
        hi = cum[ii]
        seg = total / B
        k = np.arange(B)
        assert np.all(hi >= k * seg - 1e-6 * total) and np.all(lo <= (k + 1) * seg + 1e-6 * total)
        np.testing.assert_allclose(ww, (leaf[ii] / pmin) ** -0.4, rtol=1e-5)
        np.add.at(counts, ii, 1)
    # stratified sampling makes bin counts nearly deterministic: compare 64-leaf bins
    expected = leaf / total * B * 200
    nb = C // 64
    cb = counts[:nb * 64].reshape(nb, 64).sum(1)
    eb = expected[:nb * 64].reshape(nb, 64).sum(1)
    rel = np.abs(cb - eb).sum() / eb.sum()
    assert rel < 0.03, rel


def test_sample_glob_override_sharded(cuda):
    """glob = (global pmin, shard scale) changes only the IS weights, not the indices;
    ShardedSampling at world 1 reproduces plain sampling exactly."""
    from apex_amd.engine.hbm_replay import HBMReplay
    from apex_amd.parallel.sharded import ShardedSampling

    C = 5000
    rp = HBMReplay(C, n_envs=8, device=cuda, alpha=1.0)
    pr = torch.rand(C, device=cuda) + 0.2
    rp.write_priorities(torch.arange(C, dtype=torch.int32, device=cuda), pr, dedup=False)
    rp.filled.fill_(C)
    B = 128
    ctr = torch.zeros(1, dtype=torch.int64, device=cuda)
    i0, w0 = torch.empty(B, dtype=torch.int32, device=cuda), torch.empty(B, device=cuda)
    rp.sample_indices(B, i0, w0, ctr, beta=0.4)
    sh = ShardedSampling(rp)
    glob = sh()
    i1, w1 = torch.empty_like(i0), torch.empty_like(w0)
    rp.sample_indices(B, i1, w1, ctr, beta=0.4, glob=glob)
    assert torch.equal(i0, i1)
    torch.testing.assert_close(w1, w0, rtol=1e-6, atol=0)
    forced = torch.tensor([0.1, 2.5], device=cuda)
    rp.sample_indices(B, i1, w1, ctr, beta=0.4, glob=forced)
    assert torch.equal(i0, i1)
    leaf = rp.leaf_sum[i1.long()]
    torch.testing.assert_close(w1, 2.5 * (leaf / 0.1) ** -0.4, rtol=1e-5, atol=0)


def test_gather_transitions(cuda):
    from apex_amd.engine.hbm_replay import HBMReplay

    rp = HBMReplay(512, n_envs=4, device=cuda)
    g = torch.Generator(device="cpu").manual_seed(0)
    rp.frames.copy_(torch.randint(0, 256, rp.frames.shape, generator=g, dtype=torch.uint8).to(cuda))
    F = rp.frame_capacity
    rp.s_ids.copy_(torch.randint(0, F, (512, 4), generator=g, dtype=torch.int32).to(cuda))
    rp.s2_ids.copy_(torch.randint(0, F, (512, 4), generator=g, dtype=torch.int32).to(cuda))
    rp.action.copy_(torch.randint(0, 18, (512,), generator=g, dtype=torch.int32).to(cuda))
    rp.reward.copy_(torch.randn(512, generator=g).to(cuda))
    rp.done.copy_((torch.rand(512, generator=g) < 0.1).float().to(cuda))
    idx = torch.randint(0, 512, (64,), generator=g, dtype=torch.int32).to(cuda)
    s = torch.empty(64, 4, 84, 84, dtype=torch.uint8, device=cuda)
    s2 = torch.empty_like(s)
    a = torch.empty(64, dtype=torch.int32, device=cuda)
    r = torch.empty(64, device=cuda)
    d = torch.empty(64, device=cuda)
    rp.gather(idx, s, s2, a, r, d)
    il = idx.long()
    ref_s = rp.frames[rp.s_ids[il].long()].view(64, 4, 84, 84)
    ref_s2 = rp.frames[rp.s2_ids[il].long()].view(64, 4, 84, 84)
    assert torch.equal(s, ref_s) and torch.equal(s2, ref_s2)
    assert torch.equal(a, rp.action[il])
    assert torch.equal(r, rp.reward[il]) and torch.equal(d, rp.done[il])


def test_large_tree_levels(cuda):
    """2^21-leaf (reference replay size 2M) tree: 4 levels, sums exact vs fp64."""
    from apex_amd.engine.hbm_replay import HBMReplay

    C = 2_000_000
    rp = HBMReplay(C, n_envs=256, device=cuda, alpha=0.6, frame_capacity=4096)
    assert len(rp.level_sizes) == 5
    idx = torch.arange(0, C, 3, dtype=torch.int32, device=cuda)
    pr = torch.rand(idx.numel(), device=cuda) + 0.05
    rp.write_priorities(idx, pr, dedup=False)
    leaf = rp.leaf_sum.double()
    assert math.isclose(rp.total_priority(), float(leaf.sum()), rel_tol=1e-10)


@pytest.mark.parametrize("log2c", [20, 24])
def test_large_tree_sampling_distribution(cuda, log2c):
    """2^20 / 2^24 leaves: stratified proportional sampling matches the leaf masses
    (chi-square over 256 equal-mass-index bins)."""
    from apex_amd.engine.hbm_replay import HBMReplay

    C = 1 << log2c
    rp = HBMReplay(C, n_envs=256, device=cuda, alpha=1.0, frame_capacity=4096)  # tree only: no frame ring
    g = torch.Generator(device=cuda).manual_seed(log2c)
    pr = torch.rand(C, device=cuda, generator=g) ** 4 + 1e-3  # skewed masses
    rp.write_priorities(torch.arange(C, dtype=torch.int32, device=cuda), pr, dedup=False)
    rp.filled.fill_(C)
    B, rounds, bins = 512, 400, 256
    out_i = torch.empty(B, dtype=torch.int32, device=cuda)
    out_w = torch.empty(B, dtype=torch.float32, device=cuda)
    counts = torch.zeros(bins, dtype=torch.float64, device=cuda)
    for c in range(rounds):
        rp.sample_indices(B, out_i, out_w, torch.tensor([c], dtype=torch.int64, device=cuda), beta=0.4)
        counts += torch.bincount(out_i.long() * bins // C, minlength=bins).double()
    leaf = rp.leaf_sum.double()
    expected = leaf.view(bins, -1).sum(1) / leaf.sum() * B * rounds
    chi2 = float(((counts - expected) ** 2 / expected).sum())
    # stratified sampling is far tighter than multinomial: chi2 well under its dof (255)
    assert chi2 < 255, chi2
    assert math.isclose(rp.total_priority(), float(leaf.sum()), rel_tol=1e-9)


def test_interleaved_sample_update_keeps_tree_consistent(cuda):
    """Learner-style interleaving: sample, then write new priorities for the sampled
    (duplicate-containing) indices, repeatedly; every level stays the exact sum of its
    children and the min tree the min of the leaves."""
    from apex_amd.engine.hbm_replay import HBMReplay

    C = 1 << 18
    rp = HBMReplay(C, n_envs=256, device=cuda, alpha=0.6, frame_capacity=4096)
    g = torch.Generator(device=cuda).manual_seed(5)
    rp.write_priorities(torch.arange(C, dtype=torch.int32, device=cuda), torch.rand(C, device=cuda, generator=g) + 0.01,
                        dedup=False)
    rp.filled.fill_(C)
    B = 512
    out_i = torch.empty(B, dtype=torch.int32, device=cuda)
    out_w = torch.empty(B, dtype=torch.float32, device=cuda)
    for c in range(50):
        rp.sample_indices(B, out_i, out_w, torch.tensor([c], dtype=torch.int64, device=cuda), beta=0.4)
        rp.write_priorities(out_i, torch.rand(B, device=cuda, generator=g) * 5 + 1e-3, dedup=True)
    torch.cuda.synchronize()
    below = rp.leaf_sum.double()
    below_min = rp.leaf_min
    for k, (s, m) in enumerate(zip(rp.node_sum, rp.node_min)):
        n = s.numel()
        pad = n * 64 - below.numel()
        want = torch.nn.functional.pad(below, (0, pad)).view(n, 64).sum(1)
        torch.testing.assert_close(s, want, rtol=1e-12, atol=1e-9)
        want_min = torch.nn.functional.pad(below_min, (0, pad), value=float("inf")).view(n, 64).min(1).values
        assert torch.equal(m, want_min), k
        below, below_min = s, m


def test_sample_api_returns_the_sampled_transitions(cuda):
    """HBMReplay.sample(): every returned column equals the transition table at the
    returned idx (actions int64 like the reference buffer, no uninitialised halves)."""
    from apex_amd.engine.hbm_replay import HBMReplay

    C = 1024
    rp = HBMReplay(C, n_envs=4, device=cuda)
    g = torch.Generator(device="cpu").manual_seed(3)
    rp.frames.copy_(torch.randint(0, 256, rp.frames.shape, generator=g, dtype=torch.uint8).to(cuda))
    F = rp.frame_capacity
    rp.s_ids.copy_(torch.randint(0, F, (C, 4), generator=g, dtype=torch.int32).to(cuda))
    rp.s2_ids.copy_(torch.randint(0, F, (C, 4), generator=g, dtype=torch.int32).to(cuda))
    rp.action.copy_(torch.randint(0, 18, (C,), generator=g, dtype=torch.int32).to(cuda))
    rp.reward.copy_(torch.randn(C, generator=g).to(cuda))
    rp.done.copy_((torch.rand(C, generator=g) < 0.1).float().to(cuda))
    idx = torch.arange(C, dtype=torch.int32, device=cuda)
    rp.write_priorities(idx, torch.rand(C, device=cuda) + 0.1)
    rp.filled.fill_(C)
    s, a, r, s2, d, w, sidx = rp.sample(256, 0.4)
    torch.cuda.synchronize()
    il = sidx.long()
    assert a.dtype == torch.int64 and torch.equal(a, rp.action[il].long())
    assert torch.equal(s, rp.frames[rp.s_ids[il].long()].view(256, 4, 84, 84))
    assert torch.equal(s2, rp.frames[rp.s2_ids[il].long()].view(256, 4, 84, 84))
    assert torch.equal(r, rp.reward[il]) and torch.equal(d, rp.done[il])
    assert bool((w > 0).all()) and bool((w <= 1.0 + 1e-6).all())


def test_frame_ring_outlives_transitions_across_wraps(cuda):
    """SURVEY §5.7 / BASELINE config 5: the transition ring (slot = step*E + e mod C) and the
    frame ring (slot = (step+1)*E + e mod F, F = C + (2n+8)E) both advance E slots per actor
    step, so a transition is always overwritten before any of its 8 frames.  After many wraps
    of both rings, every live transition (sampling mass > 0) must reference only frames
    written within the n-step window of the step that emitted it (a frame overwritten later
    would carry a much newer write step)."""
    from apex_amd.engine.apex import ApexEngine, EngineConfig
    from apex_amd.engine.learner import LearnerConfig

    E, C = 64, 16 * 64
    cfg = EngineConfig(n_envs=E, replay_capacity=C, threshold_size=C, use_graphs=False,
                       learner=LearnerConfig(batch_size=32, forward="hip"))
    eng = ApexEngine(cfg, cuda)
    rp, act = eng.replay, eng.actor
    F, n = rp.frame_capacity, cfg.learner.n_step
    assert F == C + (2 * n + 8) * E
    last_write = torch.full((F,), -10**9, dtype=torch.int64)
    last_write[:E] = -1  # reset frames (step 0 initial observations)
    emit_step = torch.full((C,), -1, dtype=torch.int64)
    steps = 12 * (F // E)  # ~12 wraps of the frame ring, ~13 of the transition ring
    for _ in range(steps):
        t = int(act.step_counter.item())
        eng.actor_step()
        torch.cuda.synchronize()
        last_write[act.new_frame.long().cpu()] = t
        emitted = act.prio.cpu() > 0
        slots = act.slot.long().cpu()
        emit_step[slots[emitted]] = t
        emit_step[slots[~emitted]] = -1  # slot reused without a transition: no mass
    live = (rp.leaf_sum.cpu() > 0).nonzero().flatten()
    assert live.numel() > C // 2
    ids = torch.cat([rp.s_ids.cpu()[live], rp.s2_ids.cpu()[live]], 1).long()  # [L, 8]
    w = last_write[ids]
    te = emit_step[live].unsqueeze(1)
    assert bool((te >= 0).all()), "live slot without a recorded emission"
    # every frame of a live transition was last written in [t_emit - n - 4, t_emit]
    assert bool((w <= te).all()), "a live transition references a frame overwritten after its emission"
    assert bool((w >= te - n - 4).all())
