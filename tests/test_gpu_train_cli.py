"""apex_amd.train (GPU-resident engine CLI): run, checkpoint, resume."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_train_cli_runs_saves_and_resumes(cuda, tmp_path):
    from apex_amd import train
    from apex_amd.models.dqn import DuelingDQN
    from apex_amd.utils.checkpoint import sidecar_path

    ck = str(tmp_path / "model.pth")
    common = ["--n-envs", "64", "--replay_buffer_size", "16384", "--threshold_size", "2048", "--bps_interval", "10",
              "--save_interval", "20", "--target_update_interval", "15", "--save-path", ck,
              "--log-dir", str(tmp_path / "runs")]
    assert train.main(common + ["--max-step", "30"]) == 0
    assert os.path.exists(ck) and os.path.exists(sidecar_path(ck))
    side = torch.load(sidecar_path(ck), map_location="cpu", weights_only=True)
    assert side["counters"]["learn_steps"] == 30
    assert int(side["step_counter"].item()) == 30
    # the checkpoint is the reference state_dict
    m = DuelingDQN.from_shapes((4, 84, 84), 18)
    m.load_state_dict(torch.load(ck, map_location="cpu", weights_only=True))
    import json

    with open(tmp_path / "runs" / "scalars.jsonl") as f:
        tags = {json.loads(line)["tag"] for line in f if line.strip()}
    assert {"learner/loss", "learner/grad_norm", "learner/BPS", "actor/frames_per_sec", "replay/size"} <= tags
    # resume continues the step count and the optimizer state
    assert train.main(common + ["--max-step", "40", "--resume", ck, "--no-tb"]) == 0
    side2 = torch.load(sidecar_path(ck), map_location="cpu", weights_only=True)
    assert side2["counters"]["learn_steps"] == 40
    assert int(side2["step_counter"].item()) == 40
    assert torch.isfinite(side2["opt_s2"]).all()
