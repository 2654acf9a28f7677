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


def _engine(dev, overlap, graphs):
    from apex_amd.engine.apex import ApexEngine, EngineConfig
    from apex_amd.engine.learner import LearnerConfig

    cfg = EngineConfig(n_envs=64, replay_capacity=4096, threshold_size=2048, overlap=overlap, use_graphs=graphs,
                       publish_param_interval=4, target_update_interval=6,
                       learner=LearnerConfig(batch_size=256, forward="hip"))
    torch.manual_seed(0)
    return ApexEngine(cfg, dev)


def test_overlapped_graphs_equal_sequential_schedule(cuda):
    eng_g = _engine(cuda, True, True)
    eng_e = _engine(cuda, True, False)
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
