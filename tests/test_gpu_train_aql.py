"""GPU AQL trainer (apex_amd.train_aql, BASELINE config 4): reference cadences (target sync
every 20 iterations incl. 0, model{it}.pth every save_interval and at the last iteration),
reference-key checkpoints, exact resume through the sidecar, loss tags."""
import json
import os

import pytest
import torch

from apex_amd import train_aql
from apex_amd.engine.aql import AQLEngine
from apex_amd.model import AQL
from apex_amd.envs import make

pytestmark = pytest.mark.gpu


def _args(tmp_path, *extra):
    return train_aql.parser().parse_args(["--env", "CartPole-v0", "--n-envs", "64", "--capacity", "20000",
                                          "--save-interval", "20", "--log-interval", "10", "--no-tb",
                                          "--save-dir", str(tmp_path), *extra])


def test_train_aql_cadence_checkpoint_resume(cuda, tmp_path):
    log = tmp_path / "log.jsonl"
    last = train_aql.train(_args(tmp_path, "--max-step", "45", "--json-log", str(log)))
    assert last["iteration"] == 44 and last["target_syncs"] == 3          # iterations 0, 20, 40
    for it in (0, 20, 40, 44):
        assert (tmp_path / f"model{it}.pth").exists() and (tmp_path / f"model{it}.pth.train.pt").exists()
    recs = [json.loads(x) for x in log.read_text().splitlines()]
    assert all(r["loss_q"] == r["loss_q"] and r["loss_proposal"] == r["loss_proposal"] for r in recs)
    sd = torch.load(tmp_path / "model44.pth", map_location="cpu", weights_only=True)
    ref_keys = list(AQL(make("CartPole-v0"), propose_sample=1, uniform_sample=50, device="cpu").state_dict())
    assert list(sd) == ref_keys

    # exact resume: a fresh engine loaded from model44 carries the same weights, Adam moments,
    # step counter and target net, and continues at iteration 45
    eng = AQLEngine(train_aql.config_from_args(_args(tmp_path)), cuda)
    train_aql.load_engine(eng, str(tmp_path / "model44.pth"), 44)
    assert eng.iterations == 45
    side = torch.load(tmp_path / "model44.pth.train.pt", map_location="cpu", weights_only=True)
    torch.testing.assert_close(eng.learner.m.cpu(), side["extra"]["adam_m"], rtol=0, atol=0)
    torch.testing.assert_close(eng.learner.step_ctr.cpu(), side["extra"]["step_ctr"], rtol=0, atol=0)
    for k, v in eng.model.state_dict().items():
        torch.testing.assert_close(v.cpu(), sd[k], rtol=0, atol=0)
    for k, v in eng.target.state_dict().items():
        torch.testing.assert_close(v.cpu(), side["target"][k], rtol=0, atol=0)
    last2 = train_aql.train(_args(tmp_path, "--max-step", "50", "--resume", "latest"))
    assert last2["iteration"] == 49
    assert (tmp_path / "model49.pth").exists()
