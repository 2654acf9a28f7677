"""GPU-engine evaluator (engine/evaluator.py) vs the reference evaluator's contract
(origin_repo/eval.py:49-96): greedy (epsilon 0) actions and UNCLIPPED rewards."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(dev, favour: int, A: int = 18):
    from apex_amd.models.dqn import DuelingDQN

    torch.manual_seed(0)
    m = DuelingDQN.from_shapes((4, 84, 84), A).to(dev)
    with torch.no_grad():
        m.advantage[2].bias.zero_()
        m.advantage[2].bias[favour] = 1e4  # Q argmax = ``favour`` for every observation
    return m


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_evaluator_greedy_and_unclipped(cuda, dtype):
    from apex_amd.engine.evaluator import GPUEvaluator

    FIRE = 1  # Atari action 1: fire, no movement (actor_kernels.hip decode_action)
    ev = GPUEvaluator(_model(cuda, FIRE), n_envs=16, n_actions=18, forward="hip", dtype=dtype, device=cuda, seed=5,
                      episode_life=False, max_episode_steps=400)
    rewards = []
    for _ in range(400):
        ev.step()
        assert bool((ev.actions == FIRE).all()), "epsilon 0: every action is the argmax"
        rewards.append(ev.reward.clone())
    torch.cuda.synchronize()
    r = torch.stack(rewards)
    assert float(r.max()) == 20.0, "a hit scores 20 game points (clipping would give 1)"
    assert bool((r % 20 == 0).all()) and bool((r >= 0).all())
    eps = ev.poll()  # every env ended at least one episode (game over or the 400-step limit)
    assert len(eps) == 16 and all(0 < n <= 400 for _, n in eps)
    assert all(ret % 20 == 0 for ret, _ in eps)
    assert ev.episodes >= 16


def test_evaluator_loads_published_weights(cuda):
    """``load`` copies the source flat buffer (+ packed copies) exactly: the greedy action
    follows the newly loaded weights."""
    from apex_amd.engine.evaluator import GPUEvaluator
    from apex_amd.models.fused import make_hip_net

    a, b = _model(cuda, 3), _model(cuda, 7)
    ev = GPUEvaluator(a, n_envs=8, n_actions=18, device=cuda)
    ev.step()
    assert bool((ev.actions == 3).all())
    src_flat = b.flatten_parameters()
    ev.load(src_flat, make_hip_net(b, "fp32"))
    ev.step()
    torch.cuda.synchronize()
    assert bool((ev.actions == 7).all())
    assert torch.equal(ev.flat, src_flat)
