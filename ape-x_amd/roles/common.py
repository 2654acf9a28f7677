"""Shared runtime for the role processes.

* :class:`RoleLayout` -- fixed rank map: replay 0, learner 1, evaluator 2 (optional,
  ``N_EVAL``), actors ``first_actor + ACTOR_ID``.  Every role derives the same world
  size from ``N_ACTORS``/``N_EVAL``, so ``init_process_group`` *is* the reference's
  connection handshake (learner.py:30-54): nobody proceeds until all roles are up.
* :func:`init_role` -- ``torch.distributed`` over gloo (host tensors: actors are CPU
  processes like the reference's) with the rendezvous store on ``REPLAY_IP``.
* :class:`ParamChannel` -- learner -> actors/evaluator weights through the
  rendezvous store as a versioned blob: "latest wins" like the origin PUB/SUB with
  CONFLATE=1 (actor.py:44), and a dead subscriber can never block the publisher.
* :class:`Heartbeat` / :func:`dead_ranks` -- liveness keys in the store; the learner
  keeps training when actors die (Ape-X tolerates lost actors).
* :func:`maybe_fault` -- ``APEX_FAULT=actor1:kill@200`` fault injection for tests.
* :class:`ChunkEncoder` -- actor-side chunk builder: frame-id dedup of LazyFrames
  stacks, so every 84x84 frame crosses the wire once (origin pickles whole stacks).
"""
from __future__ import annotations

import collections
import datetime
import os
import threading
import time

import numpy as np
import torch
import torch.distributed as dist

from . import wire

REPLAY_RANK = 0
LEARNER_RANK = 1


class RoleLayout:
    def __init__(self, n_actors: int, n_eval: int = 1):
        self.n_actors = int(n_actors)
        self.n_eval = int(n_eval)
        self.eval_rank = 2 if self.n_eval else None
        self.first_actor = 2 + self.n_eval
        self.world_size = self.first_actor + self.n_actors

    @classmethod
    def from_env(cls, environ=None) -> "RoleLayout":
        env = os.environ if environ is None else environ
        return cls(int(env.get("N_ACTORS", 1)), int(env.get("N_EVAL", 1)))

    def actor_rank(self, actor_id: int) -> int:
        if not 0 <= actor_id < self.n_actors:
            raise ValueError(f"ACTOR_ID {actor_id} outside [0, {self.n_actors})")
        return self.first_actor + actor_id

    def actor_ranks(self) -> list[int]:
        return list(range(self.first_actor, self.world_size))

    def rank_of(self, role: str, actor_id: int = 0) -> int:
        if role == "replay":
            return REPLAY_RANK
        if role == "learner":
            return LEARNER_RANK
        if role == "eval":
            if self.eval_rank is None:
                raise ValueError("layout has no evaluator (N_EVAL=0)")
            return self.eval_rank
        if role == "actor":
            return self.actor_rank(actor_id)
        raise ValueError(role)


def init_role(role: str, layout: RoleLayout, actor_id: int = 0, replay_ip: str | None = None,
              port: int | None = None, timeout_s: float = 600.0) -> int:
    rank = layout.rank_of(role, actor_id)
    ip = replay_ip or os.environ.get("REPLAY_IP", "127.0.0.1")
    port = int(port or os.environ.get("APEX_PORT", os.environ.get("MASTER_PORT", 29555)))
    dist.init_process_group("gloo", init_method=f"tcp://{ip}:{port}", rank=rank, world_size=layout.world_size,
                            timeout=datetime.timedelta(seconds=timeout_s))
    return rank


def store():
    return dist.distributed_c10d._get_default_store()


# ---------------------------------------------------------------------- params
class ParamChannel:
    KEY, VER = "apex/params", "apex/param_version"

    def __init__(self, st=None):
        self.st = st or store()

    def publish(self, flat: torch.Tensor) -> int:
        blob = wire.pack({"flat": flat.detach().float().cpu().numpy()})
        self.st.set(self.KEY, blob.tobytes())
        return int(self.st.add(self.VER, 1))

    def version(self) -> int:
        return int(self.st.add(self.VER, 0))

    def fetch(self, have: int = 0):
        """(version, flat tensor) if newer than ``have``, else (have, None)."""
        v = self.version()
        if v <= have:
            return have, None
        blob = np.frombuffer(self.st.get(self.KEY), dtype=np.uint8)
        return v, torch.from_numpy(wire.unpack(blob)["flat"].copy())

    def wait(self, have: int = 0, timeout: float = 600.0, poll: float = 0.05):
        t0 = time.time()
        while True:
            v, flat = self.fetch(have)
            if flat is not None:
                return v, flat
            if time.time() - t0 > timeout:
                raise TimeoutError("no parameters published")
            time.sleep(poll)


def model_flat(model) -> torch.Tensor:
    return torch.cat([p.detach().reshape(-1).float().cpu() for p in model.parameters()])


def load_model_flat_(model, flat: torch.Tensor) -> None:
    off = 0
    with torch.no_grad():
        for p in model.parameters():
            n = p.numel()
            p.copy_(flat[off:off + n].view_as(p))
            off += n


# ---------------------------------------------------------------------- liveness
class Heartbeat:
    def __init__(self, rank: int, interval: float = 1.0, st=None):
        self.rank, self.interval = rank, interval
        self.st = st or store()
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self):
        while not self._stop.is_set():
            try:
                self.st.set(f"apex/hb/{self.rank}", repr(time.time()))
            except Exception:  # store gone: the job is ending
                return
            self._stop.wait(self.interval)

    def stop(self, join_timeout: float = 10.0):
        """Stop and JOIN the beat thread: a daemon thread still inside a TCPStore call when the
        interpreter exits (the store's server -- the learner -- may already be gone) aborts the
        process ('terminate called without an active exception')."""
        self._stop.set()
        if self._t.is_alive() and threading.current_thread() is not self._t:
            self._t.join(join_timeout)


def dead_ranks(ranks, timeout: float = 10.0, st=None) -> list[int]:
    st = st or store()
    now, dead = time.time(), []
    for r in ranks:
        try:
            if st.check([f"apex/hb/{r}"]):
                last = float(st.get(f"apex/hb/{r}").decode())
                if now - last > timeout:
                    dead.append(r)
            else:
                dead.append(r)
        except Exception:
            dead.append(r)
    return dead


def maybe_fault(role: str, idx: int, step: int, environ=None) -> None:
    """``APEX_FAULT="<role><idx>:kill@<step>"`` (e.g. ``actor1:kill@200``): hard-exit
    this process at that step, without any cleanup (simulates a crashed node)."""
    spec = (os.environ if environ is None else environ).get("APEX_FAULT", "")
    for item in filter(None, spec.split(",")):
        who, _, what = item.partition(":")
        action, _, at = what.partition("@")
        if who == f"{role}{idx}" and action == "kill" and int(at) == step:
            os._exit(17)


# ---------------------------------------------------------------------- actor chunks
class ChunkEncoder:
    """Turns BatchStorage output into a wire chunk.  Image observations (LazyFrames)
    are sent as per-actor frame sequence ids; a frame's pixels travel only the first
    time it is referenced."""

    def __init__(self, keep: int = 512):
        self.ids: dict[int, int] = {}
        self.keep: collections.deque = collections.deque()
        self.keep_n = keep
        self.next_seq = 0
        self.pending_seq: list[int] = []
        self.pending_frames: list[np.ndarray] = []

    def _frame_id(self, f) -> int:
        key = id(f)
        seq = self.ids.get(key)
        if seq is None:
            seq = self.next_seq
            self.next_seq += 1
            self.ids[key] = seq
            self.keep.append(f)  # holding the object keeps id() unique
            if len(self.keep) > self.keep_n:
                del self.ids[id(self.keep.popleft())]
            self.pending_seq.append(seq)
            self.pending_frames.append(np.asarray(f, dtype=np.uint8).reshape(-1))
        return seq

    def stack_ids(self, obs) -> list[int]:
        return [self._frame_id(f) for f in obs.frames()]

    def encode(self, states, actions, rewards, next_states, dones, prios) -> dict:
        n = len(prios)
        out = {"a": np.asarray(actions, dtype=np.int64).reshape(n), "r": np.asarray(rewards, dtype=np.float32),
               "d": np.asarray(dones, dtype=np.float32), "prio": np.asarray(prios, dtype=np.float64)}
        if n and hasattr(states[0], "frames"):
            out["s"] = np.asarray([self.stack_ids(s) for s in states], dtype=np.int64)
            out["s2"] = np.asarray([self.stack_ids(s) for s in next_states], dtype=np.int64)
            out["seq"] = np.asarray(self.pending_seq, dtype=np.int64)
            out["frames"] = (np.stack(self.pending_frames) if self.pending_frames
                             else np.zeros((0, 1), dtype=np.uint8))
            self.pending_seq, self.pending_frames = [], []
        else:
            out["s"] = np.asarray([np.asarray(s, dtype=np.float32) for s in states], dtype=np.float32)
            out["s2"] = np.asarray([np.asarray(s, dtype=np.float32) for s in next_states], dtype=np.float32)
        return out


# ---------------------------------------------------------------------- envs / stop flag
def make_role_env(cfg, clip_rewards: bool | None = None, seed: int | None = None):
    """Atari ids get ``make_atari`` + ``wrap_atari_dqn`` (origin actor.py:56-57); any
    other registered id is built plainly (the origin roles are Atari-only)."""
    import copy

    from .. import envs

    env_cfg = copy.copy(cfg.env)
    if clip_rewards is not None:
        env_cfg.clip_rewards = int(clip_rewards)
    if "NoFrameskip" in env_cfg.env:
        env = envs.wrap_atari_dqn(envs.make_atari(env_cfg.env), env_cfg)
    else:
        env = envs.make(env_cfg.env)
    if seed is not None:
        env.seed(seed)
    return env


STOP_KEY = "apex/stop"


def request_stop(st=None) -> None:
    (st or store()).set(STOP_KEY, b"1")


def stop_requested(st=None) -> bool:
    st = st or store()
    try:
        return bool(st.check([STOP_KEY]))
    except Exception:
        return True
