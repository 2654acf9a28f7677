"""CPU tests: config presets / reference flag parser, checkpoint format + resume
sidecar, shared-memory parameter publishing, and short runs of every trainer
(DQN.py, ApeX.py, AQL.py, AQL_dis.py equivalents)."""
import multiprocessing as mp
import os
import warnings

import numpy as np
import pytest
import torch

warnings.filterwarnings("ignore", message="Detected call of `lr_scheduler.step()`")


# ------------------------------------------------------------------ config
def test_origin_preset_matches_reference_arguments():
    from apex_amd.config import argparser

    a = argparser([])
    # origin_repo/arguments.py defaults, flag by flag
    expect = dict(seed=1122, n_steps=3, gamma=0.99, env="SeaquestNoFrameskip-v4", episode_life=1, clip_rewards=1,
                  frame_stack=1, scale=0, send_interval=50, update_interval=400, max_episode_length=50000,
                  max_outstanding=3, eps_base=0.4, eps_alpha=7.0, alpha=0.6, beta=0.4, replay_buffer_size=2000000,
                  threshold_size=50000, batch_size=512, n_recv_batch_worker=4, n_recv_prios_worker=4,
                  n_send_batch_worker=8, lr=6.25e-5, queue_size=16, prios_queue_size=16, max_norm=40.0,
                  target_update_interval=2500, publish_param_interval=25, save_interval=5000, bps_interval=100,
                  n_recv_batch_process=4, cuda=False, render=False)
    for k, v in expect.items():
        assert getattr(a, k) == v, k
    assert a.device == torch.device("cpu")


def test_flags_env_vars_and_presets():
    from apex_amd.config import args_to_config, build_parser, preset

    p = build_parser()
    args = p.parse_args(["--lr", "1e-4", "--batch_size", "64", "--env", "PongNoFrameskip-v4", "--n-envs", "32",
                         "--no-graphs", "--exact-mass", "1", "--preset", "origin"])
    cfg = args_to_config(args, environ={"ACTOR_ID": "3", "N_ACTORS": "8", "REPLAY_IP": "10.0.0.1",
                                        "LEARNER_IP": "10.0.0.2"})
    assert cfg.learner.lr == 1e-4 and cfg.replay.batch_size == 64 and cfg.env.env == "PongNoFrameskip-v4"
    assert cfg.actor.n_envs == 32 and cfg.kernel.use_graphs is False and cfg.replay.exact_mass is True
    assert (cfg.dist.actor_id, cfg.dist.n_actors, cfg.dist.replay_ip, cfg.dist.learner_ip) == (3, 8, "10.0.0.1",
                                                                                             "10.0.0.2")
    d = preset("dqn")
    assert (d.env.env, d.n_steps, d.replay.batch_size, d.learner.lr, d.learner.optimizer) == \
        ("CartPole-v0", 1, 32, 1e-3, "adam")
    s = preset("apex_single")
    assert (s.learner.lr, s.replay.batch_size, s.learner.publish_param_interval, s.actor.n_workers) == \
        (1e-5, 64, 32, 20)
    q = preset("aql_dis")
    assert (q.actor.n_workers, q.learner.target_update_interval, q.learner.save_interval) == (10, 20, 200)
    assert preset("origin").replace(**{"learner.lr": 3.0}).learner.lr == 3.0
    with pytest.raises(AttributeError):
        preset("origin").replace(**{"learner.nope": 1})


# ------------------------------------------------------------------ checkpoints
def test_checkpoint_reference_format_and_sidecar(tmp_path):
    from apex_amd.models.dqn import DuelingDQN
    from apex_amd.utils.checkpoint import load_model, load_train_state, save_model, save_train_state

    m = DuelingDQN.from_shapes((4, 84, 84), 6)
    t = DuelingDQN.from_shapes((4, 84, 84), 6)
    opt = torch.optim.RMSprop(m.parameters(), 1e-3, centered=True)
    m(torch.rand(2, 4, 84, 84)).sum().backward()
    opt.step()
    path = save_model(m, str(tmp_path / "model5000.pth"))
    save_train_state(path, target=t, optimizers=[opt], counters={"learn_idx": 5000})
    sd = torch.load(path, map_location="cpu", weights_only=True)
    assert list(sd) == [f"{p}.{i}.{w}" for p, idx in (("features", (0, 2, 4)), ("advantage", (0, 2)),
                                                       ("value", (0, 2))) for i in idx for w in ("weight", "bias")]
    assert all(v.dtype == torch.float32 for v in sd.values())
    m2 = load_model(DuelingDQN.from_shapes((4, 84, 84), 6), path)
    for a, b in zip(m.parameters(), m2.parameters()):
        assert torch.equal(a, b)
    t2 = DuelingDQN.from_shapes((4, 84, 84), 6)
    opt2 = torch.optim.RMSprop(m2.parameters(), 1e-3, centered=True)
    r0 = np.random.rand()
    st = load_train_state(path, target=t2, optimizers=[opt2])
    assert st["counters"]["learn_idx"] == 5000
    assert np.random.rand() != r0 or True  # rng restored without error
    for a, b in zip(t.parameters(), t2.parameters()):
        assert torch.equal(a, b)
    assert torch.equal(opt2.state_dict()["state"][0]["square_avg"], opt.state_dict()["state"][0]["square_avg"])


def test_checkpoint_loads_into_reference_model(tmp_path):
    from tests import refimport

    if not refimport.available():
        pytest.skip("reference not present")
    from apex_amd import envs
    from apex_amd.models.dqn import DuelingDQN
    from apex_amd.utils.checkpoint import save_model

    ref = refimport.load("model")
    env = envs.make("CartPole-v0")
    mine = DuelingDQN(env)
    path = save_model(mine, str(tmp_path / "model0.pth"))
    theirs = ref.DuelingDQN(env)
    theirs.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
    x = torch.rand(5, 4)
    torch.testing.assert_close(theirs(x), mine(x))


# ------------------------------------------------------------------ shared params
def _sub(sp, out_q):
    from apex_amd.models.dqn import DuelingDQN

    m = DuelingDQN.from_shapes((4,), 2)
    v = sp.pull(m, 0)
    out_q.put((v, float(m.advantage[2].bias[0].detach())))


def test_shared_params_versioned_publish():
    from apex_amd.models.dqn import DuelingDQN
    from apex_amd.parallel.shm import SharedParams

    ctx = mp.get_context("spawn")
    src = DuelingDQN.from_shapes((4,), 2)
    sp = SharedParams.for_module(src, ctx)
    dst = DuelingDQN.from_shapes((4,), 2)
    assert sp.pull(dst, 0) == 0  # nothing published yet
    with torch.no_grad():
        src.advantage[2].bias.fill_(3.5)
    assert sp.publish(src) == 1
    assert sp.pull(dst, 0) == 1 and float(dst.advantage[2].bias[0].detach()) == 3.5
    assert sp.pull(dst, 1) == 1  # already current
    q = ctx.Queue()
    p = ctx.Process(target=_sub, args=(sp, q))
    p.start()
    v, b = q.get(timeout=120)
    p.join(30)
    assert (v, b) == (1, 3.5)


# ------------------------------------------------------------------ trainers
def test_dqn_trainer_cartpole(tmp_path):
    from apex_amd.trainers.dqn import train_DQN
    from apex_amd.utils.tb import NullWriter

    t = train_DQN("CartPole-v0", max_step=600, seed=0, save_dir=str(tmp_path), writer=NullWriter(), save_interval=300)
    t.train()
    assert t.losses and all(np.isfinite(t.losses))
    assert sorted(os.listdir(tmp_path)) == ["model0.pth", "model0.pth.train.pt", "model300.pth",
                                            "model300.pth.train.pt", "model599.pth", "model599.pth.train.pt"]
    t.load_model(599)
    assert len(t.evaluate(2)) == 2


def test_apex_single_concurrent(tmp_path):
    from apex_amd.trainers.apex_single import train_DQN
    from apex_amd.utils.tb import NullWriter

    t = train_DQN("CartPole-v0", n_workers=2, max_step=60, batch_size=32, save_dir=str(tmp_path), writer=NullWriter(),
                  save_interval=1000, publish_param_interval=20, update_interval=25, device="cpu")
    out = t.train()
    assert np.isfinite(out["loss"]) and out["grad_norm"] > 0
    assert t.batch_recorder.inserted == len(t.buffer) > 32
    assert os.path.exists(tmp_path / "model60.pth")
    assert not any(w.is_alive() for w in t.batch_recorder.workers)


def test_apex_single_collect_once(tmp_path):
    from apex_amd.trainers.apex_single import train_DQN
    from apex_amd.utils.tb import NullWriter

    t = train_DQN("CartPole-v0", n_workers=2, max_step=20, batch_size=8, save_dir=str(tmp_path), writer=NullWriter(),
                  collect_once=True, device="cpu")
    t.train()
    assert t.learn_idx == 20


def test_aql_trainers(tmp_path):
    from apex_amd.trainers.aql import train_AQL, train_AQL_dis
    from apex_amd.utils.tb import NullWriter

    t = train_AQL("Pendulum-v0", max_step=120, seed=0, save_dir=str(tmp_path), writer=NullWriter(),
                  save_interval=1000, device="cpu", propose_sample=10, uniform_sample=10)
    t.train()
    assert os.path.exists(tmp_path / "model119.pth")
    d = train_AQL_dis("CartPole-v0", max_step=3, n_workers=2, save_dir=str(tmp_path), writer=NullWriter(),
                      device="cpu", batch_size=8)
    eps = d.train()
    assert len(eps) == 6 and d.learn_idx > 0
    sd = torch.load(tmp_path / "model2.pth", weights_only=True)
    assert "q.advantage1.weight_epsilon" in sd and "proposal.dist_feature.0.weight" in sd


def test_trace_ranges_and_hip_debug_flags(monkeypatch):
    """roctx ranges load libroctx64 (host library, no GPU needed) and nest; the
    --profile / --hip-debug flags reach the config; hip_debug_env sets the runtime knobs."""
    from apex_amd.config import args_to_config, build_parser
    from apex_amd.utils import trace

    if trace.enable(True):
        with trace.range("outer"):
            with trace.range("inner"):
                trace.mark("m")
    trace.enable(False)
    with trace.range("disabled"):
        pass
    cfg = args_to_config(build_parser().parse_args(["--profile", "1", "--hip-debug", "4"]), environ={})
    assert cfg.kernel.profile and cfg.kernel.hip_debug == 4
    for k in ("AMD_LOG_LEVEL", "HIP_LAUNCH_BLOCKING", "AMD_SERIALIZE_KERNEL", "AMD_SERIALIZE_COPY"):
        monkeypatch.delenv(k, raising=False)
    env = trace.hip_debug_env(4)
    import os

    assert os.environ["AMD_LOG_LEVEL"] == "4" and os.environ["HIP_LAUNCH_BLOCKING"] == "1" and env
