"""Multi-rank GPU engines on ONE MI355X (ranks share cuda:0, gloo backend: host-staged
collectives / P2P).  RCCL needs one GPU per rank (the driver's 8-GPU run); these tests run
the real engines' multi-rank code paths end to end:

* sharded data-parallel ApexEngine, 2 ranks: replicas stay bit-identical after every
  step, and the in-kernel global-PER IS weights equal parallel/sharded.py's formula
  (global min priority, shard scale world * M_r / sum M) on the live trees;
* central ApexEngine, 2 ranks, over both transports -- HIP IPC (rings in rank 0's HBM,
  ingest inside the learner graph; parallel/ipc.py) and the torch.distributed P2P links
  (parallel/experience.py): after the stop every transition row and frame the actor
  produced is in rank 0's region of the replay;
* central over HIP IPC, 3 ranks, actor rank 2 hard-killed mid-run (APEX_FAULT): rank 0
  drops it and keeps stepping on rank 1's experience.
Children are started with the spawn method (fresh interpreters: no GPU state inherited).
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _child(fn, rank, world, port, q, env, args):
    import faulthandler
    import traceback

    os.environ.update(env)
    log_dir = os.environ.get("APEX_TEST_CHILD_LOGS")
    if log_dir:  # diagnostics: native-crash tracebacks + periodic stack dumps of every rank
        os.makedirs(log_dir, exist_ok=True)
        f = open(os.path.join(log_dir, f"{fn.__name__}_rank{rank}.log"), "w", buffering=1)
        f.write(f"rank {rank} pid {os.getpid()} started\n")
        faulthandler.enable(file=f)
        faulthandler.dump_traceback_later(30, repeat=True, file=f)
        os.environ["APEX_TEST_PROGRESS"] = f.name
    try:
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        res = fn(rank, world, *args)
        q.put((rank, res))
    except Exception:
        q.put((rank, "ERROR " + traceback.format_exc()))
    q.close()
    q.join_thread()
    os._exit(0)  # no collective teardown (a peer may be dead by design)


def _run(fn, world, args=(), env=None, timeout=240):
    """Spawn ``world`` ranks; collect the results of every rank that reports (a rank that
    dies without reporting, e.g. a fault-injected actor, is simply absent)."""
    import queue
    import time

    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_child, args=(fn, r, world, port, q, dict(env or {}), args)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    deadline = time.monotonic() + timeout
    try:
        while len(out) < world and time.monotonic() < deadline:
            try:
                r, res = q.get(timeout=1.0)
                out[r] = res
            except queue.Empty:
                if all(not p.is_alive() for i, p in enumerate(procs) if i not in out):
                    break  # every silent rank has exited
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    for r, res in out.items():
        assert not (isinstance(res, str) and res.startswith("ERROR")), f"rank {r}: {res}"
    return out, [p.exitcode for p in procs]


# ------------------------------------------------------------------ sharded DP
def _sharded_body(rank, world, steps):
    import torch.distributed as dist

    from apex_amd.engine.apex import ApexEngine, EngineConfig
    from apex_amd.engine.learner import LearnerConfig
    from apex_amd.parallel.broadcast import broadcast_flat
    from apex_amd.parallel.dp import FlatGradAllReduce

    dev = torch.device("cuda", 0)
    lc = LearnerConfig(batch_size=64, forward="hip", seed=11 + rank)
    cfg = EngineConfig(n_envs=64, replay_capacity=16384, threshold_size=4096, use_graphs=False,
                       actor_offset=rank * 64, total_actors=world * 64, seed=5 + 7919 * rank, learner=lc)
    eng = ApexEngine(cfg, dev, allreduce=FlatGradAllReduce(world), sharded=True)
    L = eng.learner
    broadcast_flat(L.flat, src=0)
    L.refresh_packed()
    L.sync_target()
    L.copy_params_to(eng.actor_flat)
    eng.fill()
    same = []
    for _ in range(steps):
        eng.train_step()
        torch.cuda.synchronize(dev)
        g = [torch.empty_like(L.flat, device="cpu") for _ in range(world)]
        dist.all_gather(g, L.flat.cpu())
        same.append(all(torch.equal(g[0], x) for x in g))
    # global-PER weights on the live trees: exchange (mass, min) and sample once
    sh = eng._sharded
    sh.exchange()
    rp = eng.replay
    B = 64
    idx = torch.empty(B, dtype=torch.int32, device=dev)
    w = torch.empty(B, dtype=torch.float32, device=dev)
    ctr = torch.full((1,), 12345, dtype=torch.int64, device=dev)
    rp.sample_indices(B, idx, w, ctr, beta=0.4, shard=sh.sample_args())
    torch.cuda.synchronize(dev)
    # plain lists: a child exits right after reporting, so no shared-memory tensors in the queue
    return {"same": same, "leaf": rp.leaf_sum[idx.long()].double().cpu().tolist(), "w": w.double().cpu().tolist(),
            "mass": float(rp.node_sum[-1][0].item()), "pmin": float(rp.node_min[-1][0].item()),
            "steps": eng.learn_steps}


def test_sharded_dp_two_ranks(cuda):
    out, codes = _run(_sharded_body, 2, (6,))
    assert codes == [0, 0]
    for r in (0, 1):
        assert all(out[r]["same"]) and len(out[r]["same"]) == 6, "DP replicas diverged"
    M = [out[r]["mass"] for r in (0, 1)]
    gmin = min(out[r]["pmin"] for r in (0, 1))
    for r in (0, 1):
        o = out[r]
        leaf, w = torch.tensor(o["leaf"], dtype=torch.float64), torch.tensor(o["w"], dtype=torch.float64)
        # tree leaves hold p^alpha: w_i = (leaf_i / global min leaf)^-beta * world * M_r / sum M
        exp = (leaf / gmin) ** -0.4 * (2 * M[r] / sum(M))
        assert torch.allclose(w, exp, rtol=2e-5, atol=0), (r, (w - exp).abs().max())


# ------------------------------------------------------------------ central (async links)
def _central_cfg(capacity=8192):
    from apex_amd.engine.apex import EngineConfig
    from apex_amd.engine.learner import LearnerConfig

    lc = LearnerConfig(batch_size=64, forward="hip")
    return EngineConfig(n_envs=64, replay_capacity=capacity, threshold_size=2048, use_graphs=True,
                        publish_param_interval=5, learner=lc)


def _progress(msg):
    p = os.environ.get("APEX_TEST_PROGRESS")
    if p:
        with open(p, "a") as f:
            f.write(msg + "\n")


def _central_body(rank, world, steps, dead_after, min_seconds=0.0, transport="ipc"):
    import time

    import torch.distributed as dist

    from apex_amd.engine.central import CentralApexEngine

    dev = torch.device("cuda", 0)
    eng = CentralApexEngine(_central_cfg(), dev, rank, world, dead_after=dead_after, heartbeat_every=0.05,
                            transport=transport)
    _progress("engine built")
    if rank != 0:
        eng.capture()
        _progress("captured")
        n = 0
        while eng.train_step():
            n += 1
            if n % 200 == 0:
                _progress(f"actor steps {n}")
        _progress(f"stopped after {n} steps")
        torch.cuda.synchronize(dev)
        rp = eng.replay  # the local mirror of this rank's region -> rank 0 (world group, for the check)
        live = (eng.actor.step_counter.item(), rp.s_ids.cpu(), rp.s2_ids.cpu(), rp.action.cpu(), rp.reward.cpu(),
                rp.done.cpu(), rp.frames.cpu())
        for t in live[1:]:
            dist.send(t, 0)
        return {"actor_steps": eng.actor_steps, "sent": eng.link.n_sent, "version": eng.param_version}
    eng.fill()
    _progress("filled")
    eng.capture()
    _progress("captured")
    t0 = time.monotonic()
    per_step = []
    dropped_at = None
    while len(per_step) < steps or time.monotonic() - t0 < min_seconds:
        eng.train_step()
        per_step.append(dict(eng.applied))
        if dropped_at is None and eng.dropped:
            dropped_at = len(per_step)
        if len(per_step) % 200 == 0:
            _progress(f"learner steps {len(per_step)} live {sorted(eng.live)}")
    torch.cuda.synchronize(dev)
    wall = time.monotonic() - t0
    _progress("closing")
    links = eng.close()
    _progress(f"closed {links}")
    res = {"links": links, "learn_steps": eng.learn_steps, "per_step": per_step, "wall": wall,
           "loss": eng.learner.stats()["loss"], "dropped_at": dropped_at}
    rp = eng.replay
    mism = {}
    for r in sorted(links["live"]):
        reg = eng.regions[r]
        C, F = reg.n_slots, reg.n_frames
        mine = [torch.empty_like(rp.s_ids[:C].cpu()), torch.empty_like(rp.s2_ids[:C].cpu()),
                torch.empty_like(rp.action[:C].cpu()), torch.empty_like(rp.reward[:C].cpu()),
                torch.empty_like(rp.done[:C].cpu()), torch.empty_like(rp.frames[:F].cpu())]
        for t in mine:
            dist.recv(t, r)
        s0, f0 = reg.slot_base, reg.frame_base
        bad = 0
        bad += int(not torch.equal(rp.s_ids[s0:s0 + C].cpu(), mine[0] + f0))
        bad += int(not torch.equal(rp.s2_ids[s0:s0 + C].cpu(), mine[1] + f0))
        bad += int(not torch.equal(rp.action[s0:s0 + C].cpu(), mine[2]))
        bad += int(not torch.equal(rp.reward[s0:s0 + C].cpu(), mine[3]))
        bad += int(not torch.equal(rp.done[s0:s0 + C].cpu(), mine[4]))
        bad += int(not torch.equal(rp.frames[f0:f0 + F].cpu(), mine[5]))
        mism[r] = bad
    res["mismatch"] = mism
    return res


def _stop_while_credit_blocked_body(rank, world, killed):
    """Rank 0 never ingests until the stop, so every live actor fills its D-packet window,
    stages one more step (its local mirror already holds it) and blocks on credit.  Rank 0
    waits until that is so -- ``sent == D`` and the heartbeat, bumped only inside the
    credit wait from then on, has moved twice -- optionally drops the killed peer, and
    stops.  The staged packet must still reach the replay."""
    import time

    import torch.distributed as dist

    from apex_amd.engine.central import CentralApexEngine

    dev = torch.device("cuda", 0)
    eng = CentralApexEngine(_central_cfg(), dev, rank, world, dead_after=1.0, heartbeat_every=0.02,
                            transport="ipc")
    if rank != 0:
        eng.capture()
        while eng.train_step():
            pass
        torch.cuda.synchronize(dev)
        rp = eng.replay
        for t in (rp.s_ids.cpu(), rp.s2_ids.cpu(), rp.action.cpu(), rp.reward.cpu(), rp.done.cpu(), rp.frames.cpu()):
            dist.send(t, 0)
        return {"actor_steps": eng.actor_steps, "sent": eng.link.n_sent}
    L = eng.links
    sent, hb = L.ctrl.view("sent"), L.ctrl.view("heartbeat")
    deadline = time.monotonic() + 120
    blocked = set()
    for r in range(1, world):
        if r in killed:
            continue
        while int(sent[r - 1]) < L.D:
            assert time.monotonic() < deadline, f"actor {r} never filled its window"
            time.sleep(0.005)
        h0 = int(hb[r - 1])
        while int(hb[r - 1]) < h0 + 2:
            assert time.monotonic() < deadline, f"actor {r} not waiting for credit"
            time.sleep(0.005)
        blocked.add(r)
    for r in killed:  # its heartbeat stops: dropped before the stop
        while r in L.live:
            assert time.monotonic() < deadline, f"dead actor {r} never dropped"
            L.check_heartbeats(every=0.0)
            time.sleep(0.05)
    consumed_before = {r: int(L.ctrl.view("consumed")[r - 1]) for r in blocked}
    links = eng.close()
    rp = eng.replay
    mism = {}
    for r in sorted(links["live"]):
        reg = eng.regions[r]
        C, F = reg.n_slots, reg.n_frames
        mine = [torch.empty_like(rp.s_ids[:C].cpu()), torch.empty_like(rp.s2_ids[:C].cpu()),
                torch.empty_like(rp.action[:C].cpu()), torch.empty_like(rp.reward[:C].cpu()),
                torch.empty_like(rp.done[:C].cpu()), torch.empty_like(rp.frames[:F].cpu())]
        for t in mine:
            dist.recv(t, r)
        s0, f0 = reg.slot_base, reg.frame_base
        bad = [n for n, a, b in (("s_ids", rp.s_ids[s0:s0 + C].cpu(), mine[0] + f0),
                                 ("s2_ids", rp.s2_ids[s0:s0 + C].cpu(), mine[1] + f0),
                                 ("action", rp.action[s0:s0 + C].cpu(), mine[2]),
                                 ("reward", rp.reward[s0:s0 + C].cpu(), mine[3]),
                                 ("done", rp.done[s0:s0 + C].cpu(), mine[4]),
                                 ("frames", rp.frames[f0:f0 + F].cpu(), mine[5])) if not torch.equal(a, b)]
        mism[r] = bad
    return {"links": links, "mismatch": mism, "blocked": sorted(blocked), "consumed_before": consumed_before}


@pytest.mark.parametrize("killed", [(), (2,)], ids=["no-drop", "dropped-peer"])
def test_central_stop_while_actor_credit_blocked_loses_nothing(cuda, killed):
    world = 3 if killed else 2
    env = {"APEX_FAULT": "actor2:kill@1"} if killed else {}
    out, codes = _run(_stop_while_credit_blocked_body, world, (killed,), env=env, timeout=200)
    o = out[0]
    assert o["blocked"] == [1] and o["consumed_before"] == {1: 0}
    assert o["links"]["live"] == [1] and set(o["links"]["dropped"]) == set(killed)
    # the reset packet + every actor step, INCLUDING the one staged while credit-blocked
    assert o["links"]["applied"][1] == o["links"]["sent"][1] == out[1]["actor_steps"] + 1 == out[1]["sent"]
    assert out[1]["actor_steps"] >= o["links"]["sent"][1] - 1 >= 3
    assert o["mismatch"] == {1: []}, o["mismatch"]
    if killed:
        assert codes[2] == 17


@pytest.mark.parametrize("transport", ["ipc", "p2p"])
def test_central_two_ranks_every_row_reaches_the_replay(cuda, transport):
    out, codes = _run(_central_body, 2, (40, 30.0, 0.0, transport))
    assert codes == [0, 0]
    o = out[0]
    assert o["learn_steps"] >= 40 and o["links"]["dropped"] == {}
    # every real packet landed: the reset-frame packet + one per actor step (fillers excluded)
    assert o["links"]["applied"][1] == out[1]["actor_steps"] + 1
    assert o["mismatch"] == {1: 0}, "rank 0's region differs from the actor's local mirror"
    assert out[1]["version"] >= 1  # conflated params reached the actor


def test_central_dead_actor_is_dropped_learner_keeps_stepping(cuda):
    # the learner runs >= 8 s so the 3 s heartbeat deadline expires during training
    out, codes = _run(_central_body, 3, (120, 3.0, 8.0), env={"APEX_FAULT": "actor2:kill@25"}, timeout=200)
    assert codes[2] == 17 and 2 not in out  # rank 2 died without reporting
    o = out[0]
    assert o["learn_steps"] >= 120
    assert set(o["links"]["dropped"]) == {2} and o["links"]["live"] == [1]
    assert o["dropped_at"] is not None and o["dropped_at"] < len(o["per_step"]), "dead actor not dropped in-run"
    # rank 1's experience kept arriving after rank 2 died
    last = o["per_step"][-1]
    mid = o["per_step"][len(o["per_step"]) // 2]
    assert last[1] > mid[1]
    assert o["mismatch"] == {1: 0}
    assert o["loss"] == o["loss"]  # finite
