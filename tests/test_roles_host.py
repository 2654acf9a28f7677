"""CPU tests of the distributed role topology (replay / learner / evaluator / actors
over gloo point-to-point + the store parameter channel), the wire format, the
frame-dedup host replay and actor fault tolerance."""
import os

import numpy as np
import pytest
import torch


def test_wire_roundtrip_and_no_objects():
    from apex_amd.roles import wire

    arrs = {"a": np.arange(5, dtype=np.int64), "f": np.random.rand(3, 4).astype(np.float32),
            "u": np.zeros((2, 7056), dtype=np.uint8), "e": np.zeros((0, 1), dtype=np.uint8)}
    out = wire.unpack(wire.pack(arrs))
    for k, v in arrs.items():
        assert out[k].dtype == v.dtype and np.array_equal(out[k], v)
    bad = wire.pack({"x": np.zeros(2)})
    # forge an object dtype in the table: must be refused
    s = bytes(bad).replace(b'"<f8"', b'"|O8"')
    with pytest.raises((ValueError, TypeError)):
        wire.unpack(np.frombuffer(s, dtype=np.uint8))


def _atari_env():
    from apex_amd import envs
    from apex_amd.config import preset

    cfg = preset("origin")
    cfg.env.env = "PongNoFrameskip-v4"
    return envs.wrap_atari_dqn(envs.make_atari(cfg.env.env), cfg.env)


def test_chunk_encoder_dedups_frames_and_host_replay_reconstructs():
    from apex_amd.replay.host_frames import HostReplay
    from apex_amd.replay.nstep import BatchStorage
    from apex_amd.roles.common import ChunkEncoder

    env = _atari_env()
    env.seed(3)
    enc = ChunkEncoder()
    rep = HostReplay(1000, 0.6, True, (4, 84, 84), n_actors=1, send_interval=20, seed=0)
    st = BatchStorage(3, 0.99)
    s = env.reset()
    kept_s, kept_s2, sent_frames, n = [], [], 0, 0
    rng = np.random.default_rng(0)
    for t in range(130):
        a = int(rng.integers(env.action_space.n))
        s2, r, d, _ = env.step(a)
        st.add(s, r, a, d, rng.random(env.action_space.n).astype(np.float32))
        s = env.reset() if d else s2
        if len(st) >= 20 or d:
            batch, prios = st.make_batch()
            st.reset()
            if len(prios) == 0:
                continue
            kept_s += [np.asarray(x) for x in batch[0]]
            kept_s2 += [np.asarray(x) for x in batch[3]]
            chunk = enc.encode(*batch, prios)
            sent_frames += len(chunk["seq"])
            n += rep.add_chunk(0, chunk)
    assert n == len(kept_s) and len(rep) == n
    # every 84x84 frame crossed the "wire" about once (not 2 x 4 times per transition)
    assert sent_frames < 1.3 * n + 8
    got_s = rep.frames[rep.s_slot[:n]].reshape(n, 4, 84, 84)
    got_s2 = rep.frames[rep.s2_slot[:n]].reshape(n, 4, 84, 84)
    assert np.array_equal(got_s, np.stack(kept_s)) and np.array_equal(got_s2, np.stack(kept_s2))
    out = rep.sample(16, 0.4)
    assert out["s"].shape == (16, 4, 84, 84) and out["w"].max() <= 1.0 + 1e-6


def test_role_layout_and_fault_spec():
    from apex_amd.roles.common import RoleLayout, maybe_fault

    lay = RoleLayout(4, 1)
    assert (lay.rank_of("replay"), lay.rank_of("learner"), lay.rank_of("eval"), lay.rank_of("actor", 3)) == (0, 1, 2, 6)
    assert lay.world_size == 7 and RoleLayout(2, 0).actor_ranks() == [2, 3]
    with pytest.raises(ValueError):
        lay.rank_of("actor", 4)
    maybe_fault("actor", 1, 5, environ={"APEX_FAULT": "actor1:kill@6"})  # not yet: no exit


def _run(tmp_path, n_actors, flags, port, env_extra=None, n_eval=1):
    from apex_amd.roles.launch import launch

    log = tmp_path / "logs"
    codes = launch(n_actors, flags, n_eval=n_eval, port=port, log_dir=str(log), env_extra=env_extra, timeout=300,
                   learner_flags=["--save-path", str(tmp_path / "model.pth"), "--no-tb"], actor_flags=["--no-tb"],
                   eval_flags=["--no-tb"])
    logs = {p.stem: p.read_text() for p in log.iterdir()}
    return codes, logs


def test_roles_end_to_end_cartpole(tmp_path):
    save = str(tmp_path / "model.pth")
    flags = ["--env", "CartPole-v0", "--threshold_size", "200", "--batch_size", "32", "--send_interval", "20",
             "--update_interval", "50", "--max-step", "60", "--publish_param_interval", "10", "--bps_interval", "30"]
    codes, logs = _run(tmp_path, 2, flags, 29641, env_extra={"APEX_DRAIN_TIMEOUT": "10"})
    assert codes["learner"] == 0 and codes["replay"] == 0, logs
    assert codes["actor0"] == 0 and codes["actor1"] == 0 and codes["eval"] == 0, logs
    assert "learner done: {'steps': 60" in logs["learner"]
    assert "replay done" in logs["replay"] and "'prio_updates': 60" in logs["replay"]
    sd = torch.load(tmp_path / "model.pth", weights_only=True)
    assert "advantage.0.weight" in sd and os.path.exists(str(tmp_path / "model.pth.train.pt"))


def test_roles_survive_actor_crash_atari(tmp_path):
    flags = ["--env", "PongNoFrameskip-v4", "--threshold_size", "400", "--batch_size", "16", "--send_interval", "50",
             "--update_interval", "100", "--max-step", "20", "--publish_param_interval", "10",
             "--replay_buffer_size", "20000"]
    codes, logs = _run(tmp_path, 2, flags, 29642, env_extra={"APEX_FAULT": "actor1:kill@250",
                                                            "APEX_DRAIN_TIMEOUT": "5"}, n_eval=0)
    assert codes["actor1"] == 17  # injected crash
    assert codes["learner"] == 0 and codes["replay"] == 0 and codes["actor0"] == 0, logs
    assert "learner done: {'steps': 20" in logs["learner"]
