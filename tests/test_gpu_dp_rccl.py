"""Direct RCCL communicator (parallel/rccl.py, csrc/comm.cpp) on one GPU.

A 1-rank process group (nccl = RCCL) is the most a 1-GPU box can host: RCCL refuses two
ranks on one device (scripts/rccl_same_device_probe.py), and the driver runs the real
multi-rank case.  These tests pin the call path: the communicator bootstrap, in-place
SUM / broadcast, and the data-parallel engine step with forced collectives (RCCL
gradient all-reduce + shard-mass slots riding the conv-gradient all-reduce) replaying
bit-identically to the same step without collectives."""
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg(cuda):
    import torch.distributed as dist

    if dist.is_initialized():
        pytest.skip("a process group already exists")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=cuda)
    yield cuda
    dist.destroy_process_group()


def test_rccl_comm_all_reduce_and_broadcast(pg):
    from apex_amd.parallel.rccl import RcclGradAllReduce

    ar = RcclGradAllReduce(pg, force=True)
    assert ar.world == 1 and ar.comm.handle
    t = torch.arange(1 << 16, dtype=torch.float32, device=pg)
    ref = t.clone()
    ar.wait(ar.start(t))
    torch.cuda.synchronize()
    assert torch.equal(t, ref)  # 1-rank SUM is the identity
    b = torch.full((1000,), 7.0, device=pg)
    ar.comm.broadcast(b, 0, ar.stream)
    torch.cuda.synchronize()
    assert torch.equal(b, torch.full_like(b, 7.0))


def _engine(dev, allreduce, force):
    from apex_amd.engine.apex import ApexEngine, EngineConfig
    from apex_amd.engine.learner import LearnerConfig

    cfg = EngineConfig(n_envs=64, replay_capacity=4096, threshold_size=2048, overlap=True,
                       publish_param_interval=4, target_update_interval=6,
                       learner=LearnerConfig(batch_size=256, forward="hip"))
    torch.manual_seed(0)
    return ApexEngine(cfg, dev, allreduce=allreduce, sharded=True, force_collectives=force)


def test_dp_engine_rccl_equals_no_collectives(pg):
    from apex_amd.parallel.dp import FlatGradAllReduce
    from apex_amd.parallel.rccl import RcclGradAllReduce

    eng_r = _engine(pg, RcclGradAllReduce(pg, force=True), True)
    eng_n = _engine(pg, FlatGradAllReduce(1), False)
    assert eng_r.learner.dp_split and eng_r.learner.grad_prefix > 0
    for eng in (eng_r, eng_n):
        eng.fill()
        eng.capture()
    for _ in range(20):
        eng_r.train_step()
        eng_n.train_step()
    torch.cuda.synchronize()
    assert torch.equal(eng_r.learner.flat, eng_n.learner.flat)
    assert torch.equal(eng_r.replay.leaf_sum, eng_n.replay.leaf_sum)
    sl = eng_r._sharded.slots
    assert sl.numel() == 2 and float(sl[0]) > 0 and float(sl[1]) > 0  # (mass, min priority) exchanged


def test_dp_one_graph_with_captured_rccl_equals_phase_graphs(pg):
    """EngineConfig.dp_graph: the learner step with both RCCL all-reduces captured inside
    one hipGraph replays bit-identically to the three phase graphs with eager RCCL."""
    from apex_amd.parallel.rccl import RcclGradAllReduce

    eng_p = _engine(pg, RcclGradAllReduce(pg, force=True), True)
    eng_g = _engine(pg, RcclGradAllReduce(pg, force=True), True)
    eng_g.cfg.dp_graph = True
    for eng in (eng_p, eng_g):
        eng.fill()
        eng.capture()
    assert eng_g._g_dp is not None and eng_p._g_dp is None
    for _ in range(20):
        eng_p.train_step()
        eng_g.train_step()
    torch.cuda.synchronize()
    assert torch.equal(eng_g.learner.flat, eng_p.learner.flat)
    assert torch.equal(eng_g.replay.leaf_sum, eng_p.replay.leaf_sum)
