"""Replay server role (origin_repo/replay.py:19-187).

``python -m apex_amd.roles.replay [arguments.py flags]`` with ``N_ACTORS`` /
``REPLAY_IP`` (it hosts the rendezvous store, so start it first).

One serving loop, no lock: a receiver thread takes complete messages from any peer
(actors and the learner) and the loop serves them in arrival order:

* actor ``PUSH``  -> insert the chunk (frame-deduplicated) with the actor-computed
  priorities, ``ACK`` back (the ack carries a stop flag at shutdown);
* learner ``SAMPLE`` -> once ``threshold_size`` transitions are stored, stratified
  PER sample + IS weights, reply ``BATCH`` (``NOT_READY`` before that);
* learner ``PRIOS`` -> priority update;
* learner ``BYE`` -> stop actors at their next push, exit.

Replies go out with ``isend`` so a busy learner never stalls the server.  A peer
whose connection fails (crashed actor) is dropped; the server keeps serving the rest.
"""
from __future__ import annotations

import os
import queue
import sys
import threading
import time

import torch
import torch.distributed as dist

from ..config import argparser
from ..replay.host_frames import HostReplay
from . import wire
from .common import LEARNER_RANK, Heartbeat, RoleLayout, init_role, make_role_env, request_stop


class ReplayServer:
    """Gloo only progresses a receive inside ``wait()``, so a dedicated receiver thread
    blocks on an any-source header receive (then the payload from that sender) and
    hands complete messages to the serving loop through a queue."""

    def __init__(self, cfg, layout: RoleLayout, replay: HostReplay, log_every: float = 10.0):
        self.cfg, self.layout, self.replay = cfg, layout, replay
        self.live = set(layout.actor_ranks()) | {LEARNER_RANK}
        self.inbox: queue.Queue = queue.Queue(maxsize=256)
        self.pending_sends: list = []
        self.recv_errors = 0
        self.stopping = False
        self.log_every = log_every
        self.stats = {"pushes": 0, "samples": 0, "prio_updates": 0, "not_ready": 0}
        self.bye_time = None
        self._rx = threading.Thread(target=self._receiver, daemon=True)

    def _receiver(self):
        h = torch.zeros(wire.HEADER_LEN, dtype=torch.int64)
        while True:
            try:
                src = dist.recv(h, tag=wire.TAG_REQ)  # any source
                hl = h.tolist()
                arrays = wire.recv_payload(src, hl[1], wire.TAG_REQ) if hl[1] > 0 else None
            except RuntimeError:  # a peer's connection broke (crashed actor)
                self.recv_errors += 1
                time.sleep(0.01)
                continue
            self.inbox.put((src, hl, arrays))
            if hl[0] == wire.BYE and src == LEARNER_RANK and not (self.live - {LEARNER_RANK}):
                return

    def _reply(self, dst, kind, arrays=None, *args):
        self.pending_sends += wire.isend_msg(dst, kind, arrays, *args, tag=wire.TAG_REP)
        if len(self.pending_sends) > 64:
            self._drain_sends(32)

    def _drain_sends(self, keep=0):
        while len(self.pending_sends) > keep:
            w, _ = self.pending_sends.pop(0)
            try:
                w.wait()
            except RuntimeError:
                pass

    def handle(self, src: int, h: list, arrays) -> None:
        kind = h[0]
        if kind == wire.PUSH:
            actor = src - self.layout.first_actor
            self.replay.add_chunk(actor, arrays)
            self.stats["pushes"] += 1
            self._reply(src, wire.ACK, None, int(self.stopping))
        elif kind == wire.SAMPLE:
            B, beta = int(h[2]), h[3] / 1e6
            if len(self.replay) < max(self.cfg.replay.threshold_size, B):
                self.stats["not_ready"] += 1
                self._reply(src, wire.NOT_READY, None, len(self.replay))
            else:
                self.stats["samples"] += 1
                self._reply(src, wire.BATCH, self.replay.sample(B, beta), len(self.replay))
        elif kind == wire.PRIOS:
            self.replay.update_priorities(arrays["idx"], arrays["prio"])
            self.stats["prio_updates"] += 1
        elif kind == wire.BYE:
            self.live.discard(src)
            if src == LEARNER_RANK:
                self.stopping = True
                self.bye_time = time.time()
                request_stop()

    def serve(self, max_seconds: float | None = None, drain_timeout: float = 30.0) -> dict:
        self._rx.start()
        t0 = last_log = time.time()
        pushed0 = 0
        while True:
            try:
                src, h, arrays = self.inbox.get(timeout=0.1)
                self.handle(src, h, arrays)
            except queue.Empty:
                pass
            now = time.time()
            if now - last_log > self.log_every:
                fps = (self.replay.pushed - pushed0) / (now - last_log)
                print(f"Buffer Size / transitions/s: {len(self.replay)} / {fps:.1f}", flush=True)
                last_log, pushed0 = now, self.replay.pushed
            # shutdown: the learner said bye; wait (bounded) for every live actor to be
            # told at its next push and say bye itself
            if self.bye_time is not None and (not self.live or now - self.bye_time > drain_timeout):
                break
            if max_seconds is not None and now - t0 > max_seconds:
                break
        self._drain_sends()
        self.stats["size"] = len(self.replay)
        self.stats["unresponsive_peers"] = sorted(self.live)
        self.stats["recv_errors"] = self.recv_errors
        return self.stats


def obs_layout(env):
    shape = tuple(env.observation_space.shape)
    return len(shape) == 3, shape


def main(argv=None):
    args = argparser(argv)
    cfg = args.config
    layout = RoleLayout.from_env()
    init_role("replay", layout, replay_ip=cfg.dist.replay_ip)
    hb = Heartbeat(0)
    env = make_role_env(cfg)
    frame_mode, shape = obs_layout(env)
    replay = HostReplay(cfg.replay.replay_buffer_size, cfg.replay.alpha, frame_mode, shape, layout.n_actors,
                        cfg.actor.send_interval, cfg.replay.exact_mass, seed=cfg.seed)
    stats = ReplayServer(cfg, layout, replay).serve(drain_timeout=float(os.environ.get("APEX_DRAIN_TIMEOUT", 30)))
    print("replay done:", stats, flush=True)
    hb.stop()
    # the receiver thread may still sit in a blocking receive: leave without tearing
    # the process group down (peers are gone or told to stop)
    sys.stdout.flush()
    os._exit(0)


if __name__ == "__main__":
    main()
