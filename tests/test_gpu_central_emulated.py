"""The central learner with emulated actor links (engine/central.py ``emulate_links``,
parallel/ipc.py EmulatedActorLinks) on one MI355X -- the one-GPU model of rank 0's load at
N = R + 1 GPUs that ``bench.py --emulate-links R`` times: every packet the emulated links
pushed is applied (links complete), every row counts in the fill counter, the priority tree
stays consistent under the batched ingest writes, and the learner trains throughout."""
import pytest
import torch

from tests.test_gpu_multirank import _run

pytestmark = pytest.mark.gpu


def _emu_body(rank, world, R, steps):
    from apex_amd.engine.apex import EngineConfig
    from apex_amd.engine.central import CentralApexEngine
    from apex_amd.engine.learner import LearnerConfig

    cfg = EngineConfig(n_envs=64, replay_capacity=R * 8192, threshold_size=4096,
                       learner=LearnerConfig(batch_size=64, forward="hip"))
    eng = CentralApexEngine(cfg, torch.device("cuda", 0), emulate_links=R)
    eng.fill(timeout=120)
    eng.capture()
    for _ in range(steps):
        eng.train_step()
    torch.cuda.synchronize()
    st = eng.close()
    rp = eng.replay
    leaves = float(rp.leaf_sum.double().sum())
    root = float(rp.node_sum[-1][0])
    return {"applied": st["applied"], "sent": st["sent"], "dropped": st["dropped"], "live": st["live"],
            "filled": int(rp.filled.item()), "steps": int(eng.learner.step_counter.item()), "root": root,
            "leaves": leaves, "loss": eng.learner.stats()["loss"]}


@pytest.mark.parametrize("R", [1, 3, 7])
def test_emulated_links_complete_and_tree_consistent(cuda, R):
    out, codes = _run(_emu_body, 1, (R, 60), timeout=240)
    assert codes == [0], out
    o = out[0]
    assert not isinstance(o, str), o
    assert o["dropped"] == {} and o["live"] == list(range(1, R + 1))
    for r in range(1, R + 1):
        assert o["applied"][r] == o["sent"][r] >= 60  # every pushed packet applied (paced: >= one per step)
    assert o["filled"] == 64 * sum(o["applied"].values())  # every emulated row is a real transition
    assert o["root"] == pytest.approx(o["leaves"], rel=1e-9)
    assert o["steps"] >= 60 and o["loss"] == o["loss"]
