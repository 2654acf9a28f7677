"""Distributed actor role (origin_repo/actor.py:18-137).

``ACTOR_ID=i N_ACTORS=N REPLAY_IP=... python -m apex_amd.roles.actor [flags]``

One process (the reference uses two: exploration + a parameter-receiver process):

* epsilon_i = eps_base^(1 + i/(N-1) * eps_alpha) (N=1 -> eps_base);
* blocks for the learner's first parameters, then refreshes them (non-blocking,
  newest version wins) every ``update_interval`` steps;
* ``act -> env.step -> BatchStorage.add``; every ``send_interval`` stored
  transitions the chunk (frame-deduplicated, with actor priorities) is pushed to the
  replay with at most ``max_outstanding`` un-acked pushes in flight (credit flow
  control as origin actor.py:105-115);
* logs ``actor/episode_reward`` / ``actor/episode_length``; stops when the replay's
  ack carries the stop flag, the store's stop key is set, or ``--max-actor-steps``.

This is the CPU/gym-style actor of the reference topology; on MI355X the throughput
path runs thousands of envs per GPU inside :class:`apex_amd.engine.ActorShard`.
"""
from __future__ import annotations

import argparse
import collections
import sys

import numpy as np
import torch
import torch.distributed as dist

from ..algo.schedules import actor_epsilon
from ..config import argparser
from ..models.dqn import DuelingDQN
from ..replay.nstep import BatchStorage
from ..utils import set_global_seeds
from ..utils.tb import NullWriter, SummaryWriter
from . import wire
from .common import (REPLAY_RANK, ChunkEncoder, Heartbeat, ParamChannel, RoleLayout, init_role, load_model_flat_,
                     make_role_env, maybe_fault, stop_requested)


def _split_argv(argv):
    extra = argparse.ArgumentParser(add_help=False)
    extra.add_argument("--max-actor-steps", type=int, default=0)
    extra.add_argument("--no-tb", action="store_true")
    return extra.parse_known_args(argv)


class Actor:
    def __init__(self, cfg, layout: RoleLayout, actor_id: int, writer=None, role="actor", epsilon=None,
                 clip_rewards=None):
        self.cfg, self.layout, self.actor_id = cfg, layout, int(actor_id)
        self.role = role
        seed = cfg.seed + self.actor_id
        set_global_seeds(seed, use_torch=True)
        self.env = make_role_env(cfg, clip_rewards=clip_rewards, seed=seed)
        self.model = DuelingDQN(self.env)
        self.storage = BatchStorage(cfg.n_steps, cfg.gamma, mode=cfg.actor.nstep_mode)
        self.encoder = ChunkEncoder()
        self.params = ParamChannel()
        self.version = 0
        self.epsilon = float(actor_epsilon(self.actor_id, layout.n_actors, cfg.actor.eps_base, cfg.actor.eps_alpha)) \
            if epsilon is None else float(epsilon)
        self.writer = writer or NullWriter()
        self.inflight: collections.deque = collections.deque()
        self.stopped = False
        self.pushed = 0

    def refresh(self, block=False) -> bool:
        if block:
            self.version, flat = self.params.wait(self.version)
        else:
            self.version, flat = self.params.fetch(self.version)
        if flat is not None:
            load_model_flat_(self.model, flat)
            return True
        return False

    # -- pushes with credit flow control ------------------------------------------
    def _wait_oldest(self):
        works, ack_hdr, ack_work = self.inflight.popleft()
        ack_work.wait()
        for w, _ in works:
            w.wait()
        if int(ack_hdr[2]) == 1:
            self.stopped = True

    def push(self):
        batch, prios = self.storage.make_batch()
        self.storage.reset()
        if len(prios) == 0:
            return
        chunk = self.encoder.encode(*batch, prios)
        works = wire.isend_msg(REPLAY_RANK, wire.PUSH, chunk)
        ack = torch.zeros(wire.HEADER_LEN, dtype=torch.int64)
        self.inflight.append((works, ack, dist.irecv(ack, REPLAY_RANK, tag=wire.TAG_REP)))
        self.pushed += len(prios)
        while len(self.inflight) > self.cfg.actor.max_outstanding:
            self._wait_oldest()

    def close(self):
        try:
            while self.inflight:
                self._wait_oldest()
            wire.send_msg(REPLAY_RANK, wire.BYE)
        except RuntimeError:  # replay already gone at shutdown
            pass

    def run(self, max_steps: int = 0):
        cfg = self.cfg
        self.refresh(block=True)
        print(f"[{self.role} {self.actor_id}] received first parameters (eps={self.epsilon:.4f})", flush=True)
        ep_r, ep_len, ep_idx, step = 0.0, 0, 0, 0
        state = self.env.reset()
        while not self.stopped:
            action, q = self.model.act(torch.as_tensor(np.asarray(state), dtype=torch.float32), self.epsilon)
            next_state, reward, done, _ = self.env.step(action)
            self.storage.add(state, reward, action, done, q)
            state = next_state
            ep_r += reward
            ep_len += 1
            step += 1
            maybe_fault(self.role, self.actor_id, step)
            if done or ep_len >= cfg.env.max_episode_length:
                state = self.env.reset()
                self.writer.add_scalar("actor/episode_reward", ep_r, ep_idx)
                self.writer.add_scalar("actor/episode_length", ep_len, ep_idx)
                ep_r, ep_len = 0.0, 0
                ep_idx += 1
            if step % cfg.actor.update_interval == 0:
                self.refresh()
                if stop_requested():
                    break
            if len(self.storage) >= cfg.actor.send_interval:
                self.push()
            if max_steps and step >= max_steps:
                break
        self.close()
        return {"steps": step, "pushed": self.pushed, "episodes": ep_idx, "version": self.version}


def main(argv=None):
    extra, rest = _split_argv(sys.argv[1:] if argv is None else argv)
    args = argparser(rest)
    cfg = args.config
    layout = RoleLayout.from_env()
    actor_id = cfg.dist.actor_id
    rank = init_role("actor", layout, actor_id, replay_ip=cfg.dist.replay_ip)
    hb = Heartbeat(rank)
    writer = NullWriter() if extra.no_tb else SummaryWriter(comment=f"-{cfg.env.env}-actor{actor_id}")
    out = Actor(cfg, layout, actor_id, writer).run(extra.max_actor_steps)
    writer.close()
    hb.stop()
    print(f"[actor {actor_id}] done: {out}", flush=True)
    return out


if __name__ == "__main__":
    main()
