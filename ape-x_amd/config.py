"""Configuration tree, reference presets and the reference flag parser.

One dataclass tree replaces the reference's argparse namespace plus per-trainer
constructor kwargs:

* :class:`EnvCfg`, :class:`ActorCfg`, :class:`ReplayCfg`, :class:`LearnerCfg`,
  :class:`DistCfg`, :class:`KernelCfg` grouped under :class:`ApexConfig`;
* presets carrying the reference defaults of every entry point
  (``origin`` = origin_repo/arguments.py:5-83, ``apex_single`` = ApeX.py:14-17,
  ``dqn`` = DQN.py:16-19, ``aql`` = AQL.py:18-29, ``aql_dis`` = AQL_dis.py:19-31);
* :func:`argparser` accepts every ``arguments.py`` flag name unchanged (plus the
  build's own flags) and the role env vars ``ACTOR_ID``, ``N_ACTORS``, ``REPLAY_IP``,
  ``LEARNER_IP`` (origin_repo/actor.py:18-25, learner.py:23-27).

``args.device`` is derived from ``--cuda`` exactly like arguments.py:80-81.
"""
from __future__ import annotations

import argparse
import copy
import dataclasses
import os
from dataclasses import dataclass, field


@dataclass
class EnvCfg:
    env: str = "SeaquestNoFrameskip-v4"
    episode_life: int = 1
    clip_rewards: int = 1
    frame_stack: int = 1
    scale: int = 0
    max_episode_length: int = 50000
    action_repeat: int = 4


@dataclass
class ActorCfg:
    send_interval: int = 50
    update_interval: int = 400
    max_outstanding: int = 3
    eps_base: float = 0.4
    eps_alpha: float = 7.0
    n_envs: int = 256                # GPU actor shard: vectorised envs per rank
    nstep_mode: str = "reference"    # "reference" | "textbook"
    n_workers: int = 20              # single-node recorder workers (batchrecorder.py)


@dataclass
class ReplayCfg:
    alpha: float = 0.6
    beta: float = 0.4
    beta_anneal_steps: float = 0.0   # 0 = fixed beta (origin replay.py:178); >0 anneal to 1
    replay_buffer_size: int = 2_000_000
    threshold_size: int = 50_000
    batch_size: int = 512
    n_recv_batch_worker: int = 4
    n_recv_prios_worker: int = 4
    n_send_batch_worker: int = 8
    exact_mass: bool = False         # False reproduces the exclusive-end mass
    topology: str = "central"        # "central" | "sharded"


@dataclass
class LearnerCfg:
    lr: float = 6.25e-5
    optimizer: str = "rmsprop"       # "rmsprop" (centered) | "adam"
    rms_alpha: float = 0.95
    rms_eps: float = 1.5e-7
    centered: bool = True
    queue_size: int = 16
    prios_queue_size: int = 16
    max_norm: float = 40.0
    target_update_interval: int = 2500
    publish_param_interval: int = 25
    save_interval: int = 5000
    bps_interval: int = 100
    n_recv_batch_process: int = 4
    lr_step_size: int = 0            # StepLR (0 = off)
    lr_gamma: float = 1.0
    max_step: int = 0                # 0 = run forever (origin learner)


@dataclass
class DistCfg:
    backend: str = "auto"            # "nccl" (= RCCL on ROCm) when GPUs, else "gloo"
    master_addr: str = "127.0.0.1"
    master_port: int = 29500
    replay_ip: str = "127.0.0.1"
    learner_ip: str = "127.0.0.1"
    actor_id: int = 0
    n_actors: int = 1
    heartbeat_interval: float = 1.0
    heartbeat_timeout: float = 30.0
    allreduce_bucket_mb: float = 4.0


@dataclass
class KernelCfg:
    forward: str = "hip"             # "hip" (MFMA kernels) | "torch" (PyTorch modules)
    dtype: str = "fp32"              # "fp32" (reference precision, learner.py:139-145) | "bf16" (opt-in)
    use_graphs: bool = True
    profile: bool = False            # roctx ranges around the engine phases (utils.trace)
    hip_debug: int = 0               # >0: AMD_LOG_LEVEL=<n> + blocking/serialised launches


@dataclass
class ApexConfig:
    seed: int = 1122
    n_steps: int = 3
    gamma: float = 0.99
    cuda: bool = False
    render: bool = False
    env: EnvCfg = field(default_factory=EnvCfg)
    actor: ActorCfg = field(default_factory=ActorCfg)
    replay: ReplayCfg = field(default_factory=ReplayCfg)
    learner: LearnerCfg = field(default_factory=LearnerCfg)
    dist: DistCfg = field(default_factory=DistCfg)
    kernel: KernelCfg = field(default_factory=KernelCfg)

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    def replace(self, **kw) -> "ApexConfig":
        """Copy with dotted overrides, e.g. ``replace(**{"learner.lr": 1e-4})``."""
        out = copy.deepcopy(self)
        for k, v in kw.items():
            set_path(out, k, v)
        return out


def set_path(cfg, path: str, value) -> None:
    obj = cfg
    parts = path.split(".")
    for p in parts[:-1]:
        obj = getattr(obj, p)
    if not hasattr(obj, parts[-1]):
        raise AttributeError(f"unknown config field {path!r}")
    setattr(obj, parts[-1], value)


# ---------------------------------------------------------------------- presets
def _origin() -> ApexConfig:
    return ApexConfig()


def _apex_single() -> ApexConfig:
    # ApeX.py:14-17, 37-39: RMSprop lr 1e-5 + StepLR(1000, .99), batch 64, 1e6 buffer,
    # beta annealed over 1000 learner steps, publish every 32, 20 workers, max_step 1e5.
    c = ApexConfig(seed=0)
    c.env.env = "MountainCar-v0"
    c.replay = ReplayCfg(replay_buffer_size=1_000_000, batch_size=64, beta_anneal_steps=1000, threshold_size=64)
    c.learner = LearnerCfg(lr=1e-5, publish_param_interval=32, lr_step_size=1000, lr_gamma=0.99, max_step=100_000)
    c.actor.n_workers = 20
    return c


def _dqn() -> ApexConfig:
    # DQN.py:16-41 (n=1, Adam 1e-3, StepLR(1000,.99), PER(1e5,.6), eps 1 -> .01 over 500, no clip).
    c = ApexConfig(seed=0, n_steps=1)
    c.env.env = "CartPole-v0"
    c.replay = ReplayCfg(replay_buffer_size=100_000, batch_size=32, beta_anneal_steps=1000, threshold_size=32)
    c.learner = LearnerCfg(lr=1e-3, optimizer="adam", max_norm=0.0, target_update_interval=1000, save_interval=10_000,
                           lr_step_size=1000, lr_gamma=0.99, max_step=100_000)
    return c


def _aql() -> ApexConfig:
    # AQL.py:18-49: Pendulum, Adam 1e-4 x2 + cosine, batch 32, target 1000, save 1e4, n=1.
    c = ApexConfig(seed=0, n_steps=1)
    c.env.env = "Pendulum-v0"
    c.replay = ReplayCfg(replay_buffer_size=100_000, batch_size=32, threshold_size=32)
    c.learner = LearnerCfg(lr=1e-4, optimizer="adam", target_update_interval=1000, save_interval=10_000,
                           max_step=1_000_000)
    return c


def _aql_dis() -> ApexConfig:
    # AQL_dis.py:19-53: CartPole, Adam 1e-3 x2, batch 32, target 20 / save 200 (outer iters), 10 workers.
    c = ApexConfig(seed=0, n_steps=1)
    c.env.env = "CartPole-v0"
    c.replay = ReplayCfg(replay_buffer_size=10_000_000, batch_size=32, threshold_size=32)
    c.learner = LearnerCfg(lr=1e-3, optimizer="adam", target_update_interval=20, save_interval=200,
                           publish_param_interval=5, max_step=1_000_000)
    c.actor.n_workers = 10
    return c


PRESETS = {"origin": _origin, "apex_single": _apex_single, "dqn": _dqn, "aql": _aql, "aql_dis": _aql_dis}


def preset(name: str = "origin") -> ApexConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown preset {name!r}; choose from {sorted(PRESETS)}")
    return PRESETS[name]()


# ---------------------------------------------------------------------- flag parser
# (flag, dotted config path, type) for every origin_repo/arguments.py flag, in order.
REFERENCE_FLAGS = [
    ("seed", "seed", int), ("n_steps", "n_steps", int), ("gamma", "gamma", float),
    ("env", "env.env", str), ("episode_life", "env.episode_life", int), ("clip_rewards", "env.clip_rewards", int),
    ("frame_stack", "env.frame_stack", int), ("scale", "env.scale", int),
    ("send_interval", "actor.send_interval", int), ("update_interval", "actor.update_interval", int),
    ("max_episode_length", "env.max_episode_length", int), ("max_outstanding", "actor.max_outstanding", int),
    ("eps_base", "actor.eps_base", float), ("eps_alpha", "actor.eps_alpha", float),
    ("alpha", "replay.alpha", float), ("beta", "replay.beta", float),
    ("replay_buffer_size", "replay.replay_buffer_size", int), ("threshold_size", "replay.threshold_size", int),
    ("batch_size", "replay.batch_size", int), ("n_recv_batch_worker", "replay.n_recv_batch_worker", int),
    ("n_recv_prios_worker", "replay.n_recv_prios_worker", int),
    ("n_send_batch_worker", "replay.n_send_batch_worker", int),
    ("lr", "learner.lr", float), ("queue_size", "learner.queue_size", int),
    ("prios_queue_size", "learner.prios_queue_size", int), ("max_norm", "learner.max_norm", float),
    ("target_update_interval", "learner.target_update_interval", int),
    ("publish_param_interval", "learner.publish_param_interval", int),
    ("save_interval", "learner.save_interval", int), ("bps_interval", "learner.bps_interval", int),
    ("n_recv_batch_process", "learner.n_recv_batch_process", int),
]

# build-only flags (dashed spelling so they never collide with the reference's)
EXTRA_FLAGS = [
    ("n-envs", "actor.n_envs", int), ("nstep-mode", "actor.nstep_mode", str), ("n-workers", "actor.n_workers", int),
    ("exact-mass", "replay.exact_mass", int), ("topology", "replay.topology", str),
    ("beta-anneal-steps", "replay.beta_anneal_steps", float),
    ("optimizer", "learner.optimizer", str), ("max-step", "learner.max_step", int),
    ("lr-step-size", "learner.lr_step_size", int), ("lr-gamma", "learner.lr_gamma", float),
    ("backend", "dist.backend", str), ("master-port", "dist.master_port", int),
    ("heartbeat-timeout", "dist.heartbeat_timeout", float),
    ("forward", "kernel.forward", str), ("dtype", "kernel.dtype", str), ("no-graphs", None, None), ("profile", "kernel.profile", int),
    ("hip-debug", "kernel.hip_debug", int),
]


def get_path(cfg, path: str):
    obj = cfg
    for p in path.split("."):
        obj = getattr(obj, p)
    return obj


def build_parser(base: ApexConfig | None = None, description: str = "Ape-X (MI355X)") -> argparse.ArgumentParser:
    base = base or preset("origin")
    p = argparse.ArgumentParser(description=description)
    p.add_argument("--preset", type=str, default=None, choices=sorted(PRESETS),
                   help="start from a reference preset before applying flags")
    for flag, path, typ in REFERENCE_FLAGS:
        p.add_argument(f"--{flag}", type=typ, default=None, help=f"default {get_path(base, path)!r}")
    p.add_argument("--cuda", action="store_true", default=False, help="Enables GPU training")
    p.add_argument("--render", action="store_true", default=False)
    for flag, path, typ in EXTRA_FLAGS:
        if typ is None:
            p.add_argument(f"--{flag}", action="store_true", default=False)
        else:
            p.add_argument(f"--{flag}", type=typ, default=None)
    return p


def env_overrides(cfg: ApexConfig, environ=None) -> ApexConfig:
    """Apply the reference role env vars (ACTOR_ID, N_ACTORS, REPLAY_IP, LEARNER_IP)."""
    environ = os.environ if environ is None else environ
    if "ACTOR_ID" in environ:
        cfg.dist.actor_id = int(environ["ACTOR_ID"])
    if "N_ACTORS" in environ:
        cfg.dist.n_actors = int(environ["N_ACTORS"])
    if "REPLAY_IP" in environ:
        cfg.dist.replay_ip = environ["REPLAY_IP"]
    if "LEARNER_IP" in environ:
        cfg.dist.learner_ip = environ["LEARNER_IP"]
    if "MASTER_PORT" in environ:
        cfg.dist.master_port = int(environ["MASTER_PORT"])
    return cfg


def args_to_config(args: argparse.Namespace, base: ApexConfig | None = None, environ=None) -> ApexConfig:
    if getattr(args, "preset", None):
        cfg = preset(args.preset)
    else:
        cfg = copy.deepcopy(base) if base is not None else preset("origin")
    for flag, path, _ in REFERENCE_FLAGS:
        v = getattr(args, flag)
        if v is not None:
            set_path(cfg, path, v)
    for flag, path, typ in EXTRA_FLAGS:
        v = getattr(args, flag.replace("-", "_"))
        if typ is None:
            if v:
                cfg.kernel.use_graphs = False
        elif v is not None:
            set_path(cfg, path, bool(v) if path in ("replay.exact_mass", "kernel.profile") else v)
    cfg.cuda = bool(args.cuda)
    cfg.render = bool(args.render)
    return env_overrides(cfg, environ)


def argparser(argv=None, base: ApexConfig | None = None):
    """Reference-compatible ``argparser()``: returns a flat namespace with every
    arguments.py attribute (same names and defaults), ``args.device`` and ``args.config``
    (the full :class:`ApexConfig`)."""
    import torch

    parser = build_parser(base)
    args = parser.parse_args(argv)
    cfg = args_to_config(args, base)
    cfg.cuda = bool(args.cuda and torch.cuda.is_available())
    flat = argparse.Namespace()
    for flag, path, _ in REFERENCE_FLAGS:
        setattr(flat, flag, get_path(cfg, path))
    flat.cuda = cfg.cuda
    flat.render = cfg.render
    flat.device = torch.device("cuda" if cfg.cuda else "cpu")
    flat.config = cfg
    return flat
