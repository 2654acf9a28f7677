"""Multi-process (gloo, CPU) tests of the parallel layer: DP gradient all-reduce
equivalence, versioned parameter broadcast, sharded-replay global sampling."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(fn, world, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_entry, args=(fn, r, world, port, q, args)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, res = q.get(timeout=180)
        out[r] = res
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r, res in out.items():
        if isinstance(res, BaseException) or (isinstance(res, str) and res.startswith("ERROR")):
            raise AssertionError(f"rank {r}: {res}")
    return out


def _entry(fn, rank, world, port, q, args):
    import traceback

    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        res = fn(rank, world, *args)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception:  # pragma: no cover - reported to the parent
        q.put((rank, "ERROR " + traceback.format_exc()))


# ------------------------------------------------------------------ bodies (top level: picklable)
def _allreduce_body(rank, world):
    from apex_amd.parallel.dp import FlatGradAllReduce

    g = torch.arange(10, dtype=torch.float32) * (rank + 1)
    FlatGradAllReduce(world)(g)
    g2 = torch.arange(10, dtype=torch.float32) * (rank + 1)
    FlatGradAllReduce(world, bucket_bytes=12)(g2)  # bucketed path
    return g.tolist(), g2.tolist()


def _batch(B, seed):
    g = torch.Generator().manual_seed(seed)
    s = torch.randn(B, 4, generator=g)
    s2 = torch.randn(B, 4, generator=g)
    a = torch.randint(0, 2, (B,), generator=g)
    r = torch.randn(B, generator=g)
    d = (torch.rand(B, generator=g) < 0.3).float()
    w = torch.rand(B, generator=g) + 0.5
    return s, a, r, s2, d, w


def _dp_grads(model, tgt, batch):
    from apex_amd.algo.losses import compute_loss_device

    model.zero_grad()
    loss, _ = compute_loss_device(model, tgt, batch, 3, 0.99)
    loss.backward()
    return torch.cat([p.grad.reshape(-1) for p in model.parameters()])


def _dp_body(rank, world, B):
    from apex_amd.models.dqn import DuelingDQN
    from apex_amd.parallel.broadcast import broadcast_flat
    from apex_amd.parallel.dp import FlatGradAllReduce

    torch.manual_seed(100 + rank)  # different init on purpose: the broadcast must fix it
    model = DuelingDQN.from_shapes((4,), 2)
    flat = model.flatten_parameters()
    broadcast_flat(flat, src=0)
    tgt = DuelingDQN.from_shapes((4,), 2)
    tgt.load_state_dict(model.state_dict())
    full = _batch(B, 7)
    shard = tuple(t[rank * B // world:(rank + 1) * B // world] for t in full)
    g_dp = _dp_grads(model, tgt, shard)
    FlatGradAllReduce(world)(g_dp)
    g_full = _dp_grads(model, tgt, full)
    return (g_dp - g_full).abs().max().item(), g_full.abs().max().item(), flat[:5].tolist()


def _publish_body(rank, world):
    from apex_amd.parallel.broadcast import ParamPublisher, ParamSubscriber

    flat = torch.full((6,), float(rank))
    live = torch.zeros(6)
    pub = ParamPublisher(flat, src=0)
    sub = ParamSubscriber(pub, live)
    seen = []
    for step in range(3):
        if rank == 0:
            flat.fill_(10.0 + step)
        pub.publish()
        swapped = sub.maybe_swap()
        seen.append((swapped, sub.version, live[0].item()))
    pub.publish(version=2)  # stale version: conflate keeps the newer weights
    seen.append((sub.maybe_swap(), sub.version, live[0].item()))
    return seen


class _FakeShard:
    def __init__(self, prios):
        self.device = torch.device("cpu")
        self.node_sum = [torch.tensor([float(np.sum(prios))], dtype=torch.float64)]
        self.node_min = [torch.tensor([float(np.min(prios))], dtype=torch.float32)]


def _sharded_body(rank, world, shard_prios):
    from apex_amd.parallel.sharded import ShardedSampling

    sh = ShardedSampling(_FakeShard(shard_prios[rank]))
    glob = sh()
    return glob.tolist()


# ------------------------------------------------------------------ tests
def test_flat_grad_allreduce_mean():
    out = _spawn(_allreduce_body, 2)
    want = (torch.arange(10, dtype=torch.float32) * 1.5).tolist()
    for r in (0, 1):
        assert out[r][0] == pytest.approx(want) and out[r][1] == pytest.approx(want)


@pytest.mark.parametrize("world", [2, 4])
def test_dp_gradient_equals_single_big_batch(world):
    out = _spawn(_dp_body, world, 16)
    for r in range(world):
        err, scale, head = out[r]
        assert err <= 1e-5 * max(1.0, scale)
    for r in range(1, world):
        assert out[0][2] == pytest.approx(out[r][2])  # replicas start identical


def test_param_publisher_versions_and_conflation():
    out = _spawn(_publish_body, 2)
    for r in (0, 1):
        seen = out[r]
        assert [v for _, v, _ in seen[:3]] == [1, 2, 3]
        assert [x for _, _, x in seen[:3]] == [10.0, 11.0, 12.0]
        assert seen[3] == (False, 3, 12.0)


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_sampling_global_weights(world):
    rng = np.random.default_rng(world)
    shards = [rng.random(50 + 10 * r) * (r + 1) + 0.05 for r in range(world)]
    out = _spawn(_sharded_body, world, shards)
    M = [s.sum() for s in shards]
    pmin = min(s.min() for s in shards)
    for r in range(world):
        assert out[r][0] == pytest.approx(pmin, rel=1e-6)
        assert out[r][1] == pytest.approx(world * M[r] / sum(M), rel=1e-6)


def test_sharded_estimator_matches_single_buffer_expectation():
    """Per-shard proportional sampling + the shard scale reproduces the expectation of
    global proportional sampling with single-buffer IS weights."""
    from apex_amd.parallel.sharded import global_weights_reference

    rng = np.random.default_rng(1)
    shards = [rng.random(40) + 0.1, rng.random(60) * 4 + 0.2, rng.random(30) * 0.5 + 0.05]
    f = [rng.standard_normal(len(s)) for s in shards]
    beta = 0.4
    allp, allf = np.concatenate(shards), np.concatenate(f)
    P = allp / allp.sum()
    w_single = (len(allp) * P) ** -beta / np.max((len(allp) * P) ** -beta)
    exact = np.sum(P * w_single * allf)
    # exact expectation of the sharded estimator (mean over k DP replicas)
    k = len(shards)
    w_sh = global_weights_reference(shards, shards, beta)
    est = sum(np.sum(shards[r] / shards[r].sum() * w_sh[r] * f[r]) for r in range(k)) / k
    assert est == pytest.approx(exact, rel=1e-9)
    # and the weights of identical priorities are the single-buffer weights times the scale
    M = np.array([s.sum() for s in shards])
    for r in range(k):
        w_plain = w_sh[r] / (k * M[r] / M.sum())
        i0 = sum(len(s) for s in shards[:r])
        assert np.allclose(w_plain, w_single[i0:i0 + len(shards[r])])


def _packet(rank, k, E, FB, n_slots, n_frames):
    g = torch.Generator().manual_seed(1000 * rank + k)
    frames = torch.randint(0, 256, (E, FB), dtype=torch.uint8, generator=g)
    slot = (torch.arange(E) + k * E) % n_slots
    fslot = (torch.arange(E) + (k + 1) * E) % n_frames
    s_ids = torch.randint(0, n_frames, (E, 4), generator=g, dtype=torch.int32)
    s2_ids = torch.randint(0, n_frames, (E, 4), generator=g, dtype=torch.int32)
    a = torch.randint(0, 18, (E,), generator=g, dtype=torch.int32)
    r = torch.randn(E, generator=g)
    d = (torch.rand(E, generator=g) < 0.1).float()
    p = torch.rand(E, generator=g)
    return frames, (s_ids, s2_ids, a, r, d, p, slot.int(), fslot.int())


def _experience_body(rank, world, E, FB, steps):
    from apex_amd.parallel.experience import ExperienceReceiver, ExperienceSender, Region, apply_packet, pack_meta

    n_slots, n_frames = 4 * E, 6 * E
    if rank > 0:
        snd = ExperienceSender(E, FB, "cpu", dst=0)
        for k in range(steps):
            frames, fields = _packet(rank, k, E, FB, n_slots, n_frames)
            snd.send(frames, pack_meta(*fields, out=snd.meta.clone()))
            snd.wait()
        return "sent"
    R = world - 1
    tables = {"frames": torch.zeros(R * n_frames, FB, dtype=torch.uint8),
              "s_ids": torch.zeros(R * n_slots, 4, dtype=torch.int32),
              "s2_ids": torch.zeros(R * n_slots, 4, dtype=torch.int32),
              "action": torch.zeros(R * n_slots, dtype=torch.int32), "reward": torch.zeros(R * n_slots),
              "done": torch.zeros(R * n_slots)}
    regions = {r: Region((r - 1) * n_slots, n_slots, (r - 1) * n_frames, n_frames) for r in range(1, world)}
    rcv = ExperienceReceiver(E, FB, "cpu", range(1, world))
    bad = 0
    for k in range(steps):
        rcv.post()
        for r, (frames, meta) in rcv.take("cpu").items():
            slots, prio = apply_packet(tables, regions[r], frames, meta)
            ef, (s_ids, s2_ids, a, rew, d, p, slot, fslot) = _packet(r, k, E, FB, n_slots, n_frames)
            reg = regions[r]
            bad += int(not torch.equal(slots, (slot + reg.slot_base).int()))
            bad += int(not torch.equal(prio, p))
            bad += int(not torch.equal(tables["frames"][(fslot + reg.frame_base).long()], ef))
            sl = (slot + reg.slot_base).long()
            bad += int(not torch.equal(tables["s_ids"][sl], s_ids + reg.frame_base))
            bad += int(not torch.equal(tables["s2_ids"][sl], s2_ids + reg.frame_base))
            bad += int(not torch.equal(tables["action"][sl], a))
            bad += int(not torch.equal(tables["reward"][sl], rew) or not torch.equal(tables["done"][sl], d))
    return bad


def test_central_experience_push_regions():
    out = _spawn(_experience_body, 3, 32, 112, 7)
    assert out[0] == 0 and out[1] == "sent" and out[2] == "sent"
