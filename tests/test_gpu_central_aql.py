"""Distributed AQL_dis over HIP IPC (engine/central_aql.py) on ONE MI355X: rank 0 = the AQL
learner + replay, ranks 1..2 = actor GPUs (here: processes on the same device, gloo control
plane).  Every transition an actor pushed must be in rank 0's replay ring exactly once, at
max priority, and the learner must have trained on them -- exactly one SGD step per 32 rows
that reached the replay (the device step gate; reference AQL_dis.py:109-126,117-118,
batchrecoder_AQL.py:109-132)."""
import pytest
import torch

from tests.test_gpu_multirank import _run

pytestmark = pytest.mark.gpu


def _cfg():
    from apex_amd.engine.aql import AQLEngineConfig

    return AQLEngineConfig(env_id="CartPole-v0", n_envs=64, capacity=65536, batch_size=32, seed=3,
                           target_update_interval=4)


def _central_aql_body(rank, world, iters, transport="ipc"):
    import torch.distributed as dist

    from apex_amd.engine.central_aql import CentralAQLEngine

    dev = torch.device("cuda", 0)
    eng = CentralAQLEngine(_cfg(), dev, rank, world, heartbeat_every=0.05, transport=transport)
    if rank != 0:
        log = []
        eng.capture()  # (pushes the eager warm-up step)
        log.append(eng.pkt.cpu())
        while eng.iteration():
            torch.cuda.synchronize(dev)
            log.append(eng.pkt.cpu())
        allp = torch.stack(log)
        dist.send(torch.tensor([allp.shape[0]]), 0)
        dist.send(allp, 0)
        return {"steps": eng.actor_steps, "sent": eng.link.n_sent, "version": eng.param_version}
    import time

    eng.fill()
    a0, s0 = sum(eng.applied.values()), eng.sgd_steps()
    eng.capture()
    # the learner never waits for data (a ~0.2 ms iteration outruns the actor processes): run
    # until the links have delivered enough packets, paced a little so the actors keep up
    deadline, it = time.monotonic() + 90, 0
    while it < iters or (sum(eng.applied.values()) - a0 < iters and time.monotonic() < deadline):
        eng.iteration()
        torch.cuda.synchronize(dev)
        time.sleep(0.002)
        it += 1
    a1, s1 = sum(eng.applied.values()), eng.sgd_steps()
    cadence = {"iterations": eng.iterations, "spins": eng.spins, "syncs": list(eng.eng.target_syncs),
               "data_iterations": eng.data_iterations(), "packets_since_fill": a1 - eng._pk0 if transport == "p2p"
               else eng._packets_consumed() - eng._pk0}
    st = eng.eng.learner.stats()
    links = eng.close()
    rp = eng.eng.replay
    n = int(rp.filled.item())
    E, obs, TA = eng.E, rp.obs, rp.T * rp.adim

    def rows(st_, st2_, amu_, act_, rew_, done_):
        return torch.cat([st_, st2_, amu_, act_.view(torch.float32).unsqueeze(1), rew_.unsqueeze(1),
                          done_.unsqueeze(1)], 1)

    have = rows(rp.st[:n].cpu(), rp.st2[:n].cpu(), rp.a_mu[:n].reshape(n, TA).cpu(), rp.action[:n].cpu(),
                rp.reward[:n].cpu(), rp.done[:n].cpu())
    want = []
    for r in sorted(links["live"]):
        k = torch.empty(1, dtype=torch.int64)
        dist.recv(k, r)
        allp = torch.empty(int(k), E * (2 * obs + TA + 3))
        dist.recv(allp, r)
        for p in allp[:links["sent"][r]]:
            o = 0
            parts = []
            for w in (E * obs, E * obs, E * TA, E, E, E):
                parts.append(p[o:o + w])
                o += w
            want.append(rows(parts[0].view(E, obs), parts[1].view(E, obs), parts[2].view(E, TA),
                             parts[3].view(torch.int32), parts[4], parts[5]))
    want = torch.cat(want)
    key = lambda t: sorted(map(bytes, t.numpy().view("u1").reshape(t.shape[0], -1)))  # noqa: E731
    live_leaves = int((rp.leaf_sum[:n] > 0).sum().item())
    return {"links": links, "filled": n, "want_rows": want.shape[0], "same_rows": key(have) == key(want),
            "live_leaves": live_leaves, "learner_steps": eng.learner_steps, "K": eng.K,
            "loss_q": st["loss_q"], "sgd_steps": st["steps"], "gate_packets": a1 - a0, "gate_steps": s1 - s0,
            "cadence": cadence, "transport": eng.transport,
            "inbox": ({r: (ib.n_posted, ib.n_done) for r, ib in eng.links.inbox.items()}
                      if transport == "p2p" else None)}


@pytest.mark.parametrize("transport", ["ipc", "p2p"])
def test_central_aql_every_transition_reaches_the_learner(cuda, transport):
    """Both experience transports: the HIP IPC rings, and the torch.distributed p2p links the
    bench's preflight falls back to when IPC is unusable (here host-staged over gloo)."""
    out, codes = _run(_central_aql_body, 3, (30, transport), timeout=240)
    assert codes == [0, 0, 0]
    o = out[0]
    L = o["links"]
    assert L["dropped"] == {} and L["live"] == [1, 2]
    for r in (1, 2):  # every pushed packet applied; the actor logged exactly what it pushed
        assert L["applied"][r] == L["sent"][r] == out[r]["steps"], (L, out[r], o["inbox"])
        # (p2p: the actor's send count also holds the filler packets of the stop handshake)
        assert out[r]["sent"] == out[r]["steps"] if transport == "ipc" else out[r]["sent"] >= out[r]["steps"]
        assert out[r]["version"] >= 1  # conflated weights reached the actor
    assert o["filled"] == 64 * (L["applied"][1] + L["applied"][2]) == o["want_rows"]
    assert o["same_rows"], "rank 0's replay rows differ from what the actors pushed"
    assert o["live_leaves"] == o["filled"]  # every row inserted at (max) priority
    assert o["K"] == 2 * 64 // 32
    # the replay ratio: one SGD step per 32 rows that reached the replay (64-row packets: 2 each)
    assert o["gate_packets"] >= 30 and o["gate_steps"] == 2 * o["gate_packets"]
    assert o["loss_q"] == o["loss_q"]
    assert o["transport"] == transport
    # the reference cadence counts recorded batches (R = 2 packets each), not learner spins
    # (a spin that ingested nothing completes no iteration), and the target syncs once per
    # completed iteration i with i % 4 == 0 (AQL_dis.py:127-129)
    c = o["cadence"]
    assert c["data_iterations"] == c["packets_since_fill"] // 2 >= 10
    # (ipc: the host reads the consumed words the ingest publishes, so its count may trail
    # the GPU by the last spin)
    assert c["data_iterations"] - (1 if o["transport"] == "ipc" else 0) <= c["iterations"] <= c["data_iterations"]
    # (ipc: the paced learner outruns the actor processes -- spins that ran no SGD step do not
    # advance the cadence; the host-staged p2p links are slower, one packet per spin)
    assert c["spins"] > c["iterations"] if transport == "ipc" else c["spins"] >= c["iterations"]
    assert len(c["syncs"]) == -(-c["iterations"] // 4), c
