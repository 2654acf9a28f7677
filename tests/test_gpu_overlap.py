"""Overlapped actor/learner streams: staged actor rows + learner-side apply.

The overlapped engine runs the actor graph of step t on its own stream, concurrently
with learner step t; the actor writes its transition rows and priorities into a
staging set that the learner stream applies one step later.  These tests pin
(1) staging + apply == the direct actor write, and (2) the concurrent graphed engine
== the same schedule run sequentially (so the two streams never race)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _shard(dev, staged, mode):
    from apex_amd.engine.actor_shard import ActorShard
    from apex_amd.engine.hbm_replay import HBMReplay

    rp = HBMReplay(4096, 64, 3, 0.6, dev, seed=5)
    return rp, ActorShard(rp, 64, 18, n_step=3, gamma=0.99, seed=11, mode=mode, staged=2 if staged else 0)


@pytest.mark.parametrize("mode", ["reference", "textbook"])
def test_staged_actor_rows_match_direct_write(cuda, mode):
    rp_a, a = _shard(cuda, False, mode)
    rp_b, b = _shard(cuda, True, mode)
    g = torch.Generator(device=cuda).manual_seed(3)
    for i in range(150):  # > C/E steps: the ring wraps
        q = torch.randn(64, 18, device=cuda, generator=g)
        a.act_and_step(q)
        b.act_and_step(q, i % 2)
        b.apply_staged(i % 2)
    torch.cuda.synchronize()
    for name in ("s_ids", "s2_ids", "action", "reward", "done", "leaf_sum", "leaf_min", "filled"):
        assert torch.equal(getattr(rp_a, name), getattr(rp_b, name)), name
    for x, y in zip(rp_a.node_sum, rp_b.node_sum):
        assert torch.equal(x, y)
    assert torch.equal(rp_a.frames, rp_b.frames)
    assert torch.equal(a.step_counter, b.step_counter)


def _engine(dev, overlap, graphs, dp=False, sharded=False, actor_at="start", capacity=4096, tree_ride=True,
            draw_in_conv1=True):
    from apex_amd.engine.apex import ApexEngine, EngineConfig
    from apex_amd.engine.learner import LearnerConfig
    from apex_amd.parallel.dp import FlatGradAllReduce

    cfg = EngineConfig(n_envs=64, replay_capacity=capacity, threshold_size=2048, overlap=overlap, use_graphs=graphs,
                       publish_param_interval=4, target_update_interval=6, actor_at=actor_at,
                       learner=LearnerConfig(batch_size=256, forward="hip", tree_ride=tree_ride,
                                             draw_in_conv1=draw_in_conv1))
    torch.manual_seed(0)
    # dp: the data-parallel phase split (FC1/head all-reduce overlapping the conv backward,
    # pipelined shard-mass exchange) with a world-1 all-reduce -- same code path, 1 GPU
    return ApexEngine(cfg, dev, allreduce=FlatGradAllReduce(1) if dp else None, sharded=sharded)


@pytest.mark.parametrize("overlap,actor_at", [(True, "start"), (True, "loss"), (False, "start")])
def test_graphs_equal_sequential_schedule(cuda, overlap, actor_at):
    """The captured engine (overlap: actor graph on its own stream beside the learner graph,
    launched with the step or -- actor_at="loss" -- between the two halves of the split
    learner graph) replays exactly like the same schedule run eagerly on one stream."""
    eng_g = _engine(cuda, overlap, True, actor_at=actor_at)
    assert eng_g._split_at_loss == (actor_at == "loss")
    eng_e = _engine(cuda, overlap, False)
    for eng in (eng_g, eng_e):
        eng.fill()
    eng_g.capture()                  # 3 counted warm-up steps, run sequentially
    for _ in range(3):
        eng_e.train_step()
    for _ in range(40):              # > C/E steps after the fill: the rings wrap under overlap
        eng_g.train_step()
        eng_e.train_step()
    torch.cuda.synchronize()
    assert eng_g.learn_steps == eng_e.learn_steps == 43
    assert torch.equal(eng_g.replay.frames, eng_e.replay.frames)
    assert torch.equal(eng_g.replay.leaf_sum, eng_e.replay.leaf_sum)
    assert torch.equal(eng_g.replay.s_ids, eng_e.replay.s_ids)
    assert torch.equal(eng_g.learner.flat, eng_e.learner.flat)
    assert torch.equal(eng_g.actor_flat, eng_e.actor_flat)
    assert torch.isfinite(eng_g.learner.flat).all()


@pytest.mark.parametrize("capacity", [4096, 8192, 1 << 21])
def test_tree_riders_equal_forked_tree_stream(cuda, capacity):
    """The priority-tree write as riders of the trunk backward's launches (leaves with the FC1
    pair, level 1 with the conv3 pair, level 2 with the conv2 pair, the top walk with the gradient
    finalize -- or with the conv2 pair when only level 1 is wide) leaves the replay, the
    counters and the learner exactly as the forked tree stream does (4096: level 1 of 64 nodes;
    8192: 128; 2M: levels 1 and 2 wide, 512 nodes at level 2)."""
    engs = [_engine(cuda, True, True, capacity=capacity, tree_ride=r) for r in (True, False)]
    for eng in engs:
        eng.fill()
        eng.capture()
    assert engs[0].learner.tree_rides_used and not engs[1].learner.tree_rides_used
    for _ in range(40):
        for eng in engs:
            eng.train_step()
    torch.cuda.synchronize()
    a, b = (e.replay for e in engs)
    for name in ("leaf_sum", "leaf_min", "max_prio", "filled", "s_ids", "frames"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    for x, y in zip(a.node_sum + a.node_min, b.node_sum + b.node_min):
        assert torch.equal(x, y)
    assert torch.equal(a.owner, torch.full_like(a.owner, -1))  # every dedup claim released
    la, lb = (e.learner for e in engs)
    for name in ("flat", "step_counter", "prio", "loss", "idx", "w"):
        assert torch.equal(getattr(la, name), getattr(lb, name)), name
    # the tree is consistent: the root holds the sum of the leaves
    assert torch.allclose(a.node_sum[-1].double(), a.leaf_sum.double().sum(), rtol=1e-9)


@pytest.mark.parametrize("capacity", [4096, 1 << 21])
def test_conv1_draw_equals_sampling_launch(cuda, capacity):
    """The PER draw folded into the conv1 forward launch (each workgroup draws its samples'
    slots; problem 0's write idx / IS weights; extra workgroups scatter the staged actor rows and
    a drawn slot among them is read from the staging rows) gives exactly the batches, replay
    tables and learner of the separate sampling launch, with the actor rows staged every step."""
    engs = [_engine(cuda, True, True, capacity=capacity, draw_in_conv1=d) for d in (True, False)]
    for eng in engs:
        eng.fill()
        eng.capture()
    assert engs[0].learner.draws_in_conv1 and not engs[1].learner.draws_in_conv1
    for _ in range(40):  # 64 envs x 40 steps > 2048 free slots of the 4096 ring: staged rows overwrite drawn slots
        for eng in engs:
            eng.train_step()
    torch.cuda.synchronize()
    a, b = (e.replay for e in engs)
    for name in ("s_ids", "s2_ids", "action", "reward", "done", "leaf_sum", "max_prio", "filled"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    la, lb = (e.learner for e in engs)
    for name in ("idx", "w", "flat", "prio", "loss", "step_counter"):
        assert torch.equal(getattr(la, name), getattr(lb, name)), name
    assert la.idx.unique().numel() > la.B // 2  # real draws, not a constant slot


@pytest.mark.parametrize("overlap,sharded", [(True, False), (False, False), (True, True), (False, True)])
def test_dp_phase_graphs_equal_eager_and_single_process(cuda, overlap, sharded):
    """The data-parallel step (three phase graphs, async all-reduce slices, pipelined
    shard-mass exchange) replays exactly like its eager schedule, and its first step
    matches the single-process fused step (different grad-norm summation order only)."""
    eng_g = _engine(cuda, overlap, True, dp=True, sharded=sharded)
    eng_e = _engine(cuda, overlap, False, dp=True, sharded=sharded)
    eng_1 = _engine(cuda, overlap, False)
    assert eng_g.learner.dp_split and eng_g._dp and not eng_1._dp
    for eng in (eng_g, eng_e, eng_1):
        eng.fill()
    eng_e.train_step()
    eng_1.train_step()
    torch.cuda.synchronize()
    torch.testing.assert_close(eng_e.learner.flat, eng_1.learner.flat, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(eng_e.learner.loss, eng_1.learner.loss, rtol=1e-5, atol=1e-7)
    eng_g.train_step()                # same first step, then capture (3 counted warm-up steps)
    eng_g.capture()
    for _ in range(3):
        eng_e.train_step()
    for _ in range(30):
        eng_g.train_step()
        eng_e.train_step()
    torch.cuda.synchronize()
    assert eng_g.learn_steps == eng_e.learn_steps == 34
    assert torch.equal(eng_g.replay.leaf_sum, eng_e.replay.leaf_sum)
    assert torch.equal(eng_g.learner.flat, eng_e.learner.flat)
    assert torch.equal(eng_g.actor_flat, eng_e.actor_flat)
    assert torch.isfinite(eng_g.learner.flat).all()
