"""Learner role (origin_repo/learner.py:23-204).

``N_ACTORS=N REPLAY_IP=... python -m apex_amd.roles.learner [--cuda] [flags]``

The reference runs 1 train + 1 param-sender + 1 prio-sender + 4 batch-receiver
processes joined by torch.mp queues.  Here one process overlaps the same work:

* the next ``SAMPLE`` request is sent before the current batch is trained on, so the
  replay samples/serialises while the GPU computes (``queue_size`` prefetch depth);
* priorities go back with a non-blocking send (no ``prios.cpu()`` stall on the
  critical path beyond the one D2H copy the wire needs);
* parameters are published through the versioned store channel every
  ``publish_param_interval`` steps (conflating, like PUB/SUB + CONFLATE).

Loss/optimizer semantics follow learner.py:134-175: double-DQN n-step Huber with IS
weights, centered RMSprop(lr, .95, 1.5e-7), clip 40, target sync every 2500,
``model.pth`` every 5000 (plus the ``model.pth.train.pt`` resume sidecar), BPS log
every 100 (``learner/BPS``), ``learner/loss``, ``learner/grad_norm``.  ``--cuda``
trains on the GPU in fp32 like the reference; the fully fused MI355X learner (HBM
replay, MFMA conv kernels, hipGraphs) is :class:`apex_amd.engine.learner.DQNLearner`.
"""
from __future__ import annotations

import argparse
import collections
import os
import sys
import time

import numpy as np
import torch

from ..algo.losses import compute_loss_device, update_parameters_ex
from ..config import argparser
from ..models.dqn import DuelingDQN
from ..utils import set_global_seeds
from ..utils.checkpoint import save_model, save_train_state
from ..utils.tb import NullWriter, SummaryWriter
from . import wire
from .common import (REPLAY_RANK, Heartbeat, ParamChannel, RoleLayout, dead_ranks, init_role, make_role_env,
                     model_flat, request_stop)


def _split_argv(argv):
    extra = argparse.ArgumentParser(add_help=False)
    extra.add_argument("--max-learner-steps", type=int, default=0)
    extra.add_argument("--save-path", default="model.pth")
    extra.add_argument("--no-tb", action="store_true")
    extra.add_argument("--prefetch", type=int, default=2)
    return extra.parse_known_args(argv)


class Learner:
    def __init__(self, cfg, layout: RoleLayout, device, writer=None, save_path="model.pth", prefetch=2):
        self.cfg, self.layout, self.device = cfg, layout, torch.device(device)
        set_global_seeds(cfg.seed, use_torch=True)
        env = make_role_env(cfg)
        self.model = DuelingDQN(env).to(self.device)
        self.tgt_model = DuelingDQN(env).to(self.device)
        self.tgt_model.load_state_dict(self.model.state_dict())
        lc = cfg.learner
        self.optimizer = torch.optim.RMSprop(self.model.parameters(), lc.lr, alpha=lc.rms_alpha, eps=lc.rms_eps,
                                             centered=lc.centered)
        self.writer = writer or NullWriter()
        self.params = ParamChannel()
        self.save_path = save_path
        self.prefetch = max(1, min(int(prefetch), cfg.learner.queue_size))
        self.inflight_reqs = 0
        self.prio_sends: collections.deque = collections.deque()
        self.learn_idx = 0
        self.last = {}

    def publish(self) -> int:
        return self.params.publish(model_flat(self.model))

    def _request(self):
        beta_u = int(round(self.cfg.replay.beta * 1e6))
        wire.send_msg(REPLAY_RANK, wire.SAMPLE, None, self.cfg.replay.batch_size, beta_u)
        self.inflight_reqs += 1

    def _next_batch(self):
        while True:
            while self.inflight_reqs < self.prefetch:
                self._request()
            h, arrays = wire.recv_msg(REPLAY_RANK, tag=wire.TAG_REP)
            self.inflight_reqs -= 1
            if h[0] == wire.BATCH:
                return arrays
            time.sleep(0.05)  # NOT_READY: replay below threshold_size

    def _to_device(self, b):
        dev = self.device
        f = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev, non_blocking=True)  # noqa: E731
        s = f(b["s"]).float()
        s2 = f(b["s2"]).float()
        return (s, f(b["a"]).long(), f(b["r"]).float(), s2, f(b["d"]).float(), f(b["w"]).float())

    def step(self):
        b = self._next_batch()
        batch = self._to_device(b)
        loss, prios = compute_loss_device(self.model, self.tgt_model, batch, self.cfg.n_steps, self.cfg.gamma)
        grad_norm, l2 = update_parameters_ex(loss, self.model, self.optimizer, self.cfg.learner.max_norm)
        prios_np = prios.float().cpu().numpy().astype(np.float64)
        self.prio_sends.append(wire.isend_msg(REPLAY_RANK, wire.PRIOS, {"idx": b["idx"], "prio": prios_np}))
        while len(self.prio_sends) > self.cfg.learner.prios_queue_size:
            for w, _ in self.prio_sends.popleft():
                w.wait()
        self.learn_idx += 1
        self.last = {"loss": float(loss.detach()), "grad_norm": float(grad_norm), "grad_norm_l2": float(l2)}
        return self.last

    def run(self, max_steps: int = 0):
        lc = self.cfg.learner
        self.publish()
        t0 = time.time()
        while True:
            out = self.step()
            t = self.learn_idx
            self.writer.add_scalar("learner/loss", out["loss"], t)
            self.writer.add_scalar("learner/grad_norm", out["grad_norm"], t)
            if t % lc.target_update_interval == 0:
                print("Updating Target Network..", flush=True)
                self.tgt_model.load_state_dict(self.model.state_dict())
            if t % lc.save_interval == 0:
                print("Saving Model..", flush=True)
                self.save()
            if t % lc.publish_param_interval == 0:
                self.publish()
            if t % lc.bps_interval == 0:
                bps = lc.bps_interval / (time.time() - t0)
                dead = dead_ranks(self.layout.actor_ranks(), timeout=self.cfg.dist.heartbeat_timeout)
                print(f"Step: {t} BPS: {bps:.2f}" + (f" dead actor ranks: {dead}" if dead else ""), flush=True)
                self.writer.add_scalar("learner/BPS", bps, t)
                t0 = time.time()
            if (max_steps and t >= max_steps) or (lc.max_step and t >= lc.max_step):
                break
        self.shutdown()
        return {"steps": self.learn_idx, **self.last}

    def save(self):
        save_model(self.model, self.save_path)
        save_train_state(self.save_path, target=self.tgt_model, optimizers=[self.optimizer],
                         counters={"learn_idx": self.learn_idx})

    def shutdown(self):
        while self.prio_sends:
            for w, _ in self.prio_sends.popleft():
                w.wait()
        while self.inflight_reqs:  # drain prefetched replies
            wire.recv_msg(REPLAY_RANK, tag=wire.TAG_REP)
            self.inflight_reqs -= 1
        self.save()
        self.publish()
        request_stop()
        wire.send_msg(REPLAY_RANK, wire.BYE)


def main(argv=None):
    extra, rest = _split_argv(sys.argv[1:] if argv is None else argv)
    args = argparser(rest)
    cfg = args.config
    layout = RoleLayout.from_env()
    init_role("learner", layout, replay_ip=cfg.dist.replay_ip)
    hb = Heartbeat(1)
    writer = NullWriter() if extra.no_tb else SummaryWriter(comment=f"-{cfg.env.env}-learner")
    out = Learner(cfg, layout, args.device, writer, extra.save_path, extra.prefetch).run(extra.max_learner_steps)
    writer.close()
    hb.stop()
    print("learner done:", out, flush=True)
    return out


if __name__ == "__main__":
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    main()
