"""Single-node Ape-X trainer (reference ApeX.py:13-120).

``n_workers`` CPU actor processes (:class:`BatchRecorder`) feed a
:class:`CustomPrioritizedReplayBuffer` with actor-computed priorities; the learner
samples batch 64 with beta annealed 0.4 -> 1 over 1000 steps, runs the double-DQN
n-step loss, ``scheduler.step()`` (before the optimizer), centered RMSprop
with clip 40, then writes priorities back.  Target sync every 2500, checkpoint
``model{t}.pth`` every 5000 and at ``max_step``, weights published to the workers
every 32 learner steps.

Acting and learning run **concurrently** (the reference's ``__main__`` calls
``sampling_data()`` then ``train()`` inline, so it collects once and trains offline:
SURVEY Q7).  ``collect_once=True`` reproduces that behaviour.

The on-GPU, many-env version of this loop is :class:`apex_amd.engine.apex.ApexEngine`
(vectorised GPU actors + HBM replay + fused HIP learner); this trainer keeps the
reference's host-side structure for non-image / gym-style envs.
"""
from __future__ import annotations

import argparse
import os

import numpy as np
import torch

from .. import envs
from ..algo.losses import compute_loss, update_parameters_ex
from ..algo.schedules import beta_by_frame, step_scheduler_early
from ..models.dqn import DuelingDQN
from ..replay.buffers import CustomPrioritizedReplayBuffer
from ..utils import set_global_seeds
from ..utils.checkpoint import load_model, save_model, save_train_state
from ..utils.tb import SummaryWriter
from .batchrecorder import BatchRecorder


class train_DQN:  # noqa: N801  (reference class name)
    def __init__(self, env_id, seed=0, lr=1e-5, n_step=3, gamma=0.99, n_workers=20, max_norm=40,
                 target_update_interval=2500, save_interval=5000, batch_size=64, buffer_size=1e6, prior_alpha=0.6,
                 prior_beta=0.4, publish_param_interval=32, max_step=1e5, collect_once=False, device=None,
                 save_dir=".", writer=None, start_method="spawn", send_interval=50, update_interval=400,
                 nstep_mode="reference", max_episode_length=50000, polls_per_step=4):
        self.env = envs.make(env_id)
        self.env_id = env_id
        self.seed = int(seed)
        self.lr = lr
        self.n_step = int(n_step)
        self.gamma = gamma
        self.max_norm = max_norm
        self.target_update_interval = int(target_update_interval)
        self.save_interval = int(save_interval)
        self.publish_param_interval = int(publish_param_interval)
        self.batch_size = int(batch_size)
        self.prior_beta = prior_beta
        self.max_step = int(max_step)
        self.collect_once = collect_once
        self.save_dir = save_dir
        self.polls_per_step = polls_per_step
        set_global_seeds(self.seed, use_torch=True)
        self.buffer = CustomPrioritizedReplayBuffer(size=int(buffer_size), alpha=prior_alpha)
        self.device = torch.device(device if device is not None else ("cuda:0" if torch.cuda.is_available() else "cpu"))
        self.model = DuelingDQN(self.env).to(self.device)
        self.tgt_model = DuelingDQN(self.env).to(self.device)
        self.tgt_model.load_state_dict(self.model.state_dict())
        self.optimizer = torch.optim.RMSprop(self.model.parameters(), self.lr, alpha=0.95, eps=1.5e-7, centered=True)
        self.scheduler = torch.optim.lr_scheduler.StepLR(self.optimizer, step_size=1000, gamma=0.99)
        self.writer = writer if writer is not None else SummaryWriter(comment=f"-{self.env.unwrapped.spec.id}-learner")
        self.batch_recorder = BatchRecorder(env_id=env_id, env_seed=self.seed, n_workers=n_workers, buffer=self.buffer,
                                            n_steps=self.n_step, gamma=gamma, max_episode_length=max_episode_length,
                                            send_interval=send_interval, writer=self.writer, nstep_mode=nstep_mode,
                                            update_interval=update_interval, start_method=start_method,
                                            model=self._cpu_model())
        self.learn_idx = 0
        self.last = {}

    def _cpu_model(self):
        m = DuelingDQN(self.env)
        m.load_state_dict({k: v.cpu() for k, v in self.model.state_dict().items()})
        return m

    def beta_by_frame(self, idx):
        return beta_by_frame(idx, self.prior_beta, 1000.0)

    def _to_batch(self, s, a, r, s2, d, w):
        dev = self.device
        f32 = lambda x: torch.as_tensor(np.asarray(x, dtype=np.float32), device=dev)  # noqa: E731
        return (f32([np.asarray(o) for o in s]), torch.as_tensor(np.asarray(a), dtype=torch.int64, device=dev), f32(r),
                f32([np.asarray(o) for o in s2]), f32(d), f32(w))

    def learn_step(self):
        beta = self.beta_by_frame(self.learn_idx)
        s, a, r, s2, d, w, idxes = self.buffer.sample(self.batch_size, beta)
        batch = self._to_batch(s, a, r, s2, d, w)
        loss, prios = compute_loss(self.model, self.tgt_model, batch, self.n_step, self.gamma)
        step_scheduler_early(self.scheduler)  # Q9
        grad_norm, l2 = update_parameters_ex(loss, self.model, self.optimizer, self.max_norm)
        self.buffer.update_priorities(idxes, prios)
        self.learn_idx += 1
        self.last = {"loss": float(loss.detach()), "grad_norm": float(grad_norm), "grad_norm_l2": float(l2)}
        self.writer.add_scalar("learner/loss", self.last["loss"], self.learn_idx)
        self.writer.add_scalar("learner/grad_norm", self.last["grad_norm"], self.learn_idx)
        return self.last

    def sampling_data(self):
        """One reference recording round: every worker plays one episode."""
        return self.batch_recorder.record_batch()

    def train(self):
        rec = self.batch_recorder
        if self.collect_once:
            self.sampling_data()
        else:
            rec.start()
            rec.wait_for(self.batch_size + 1)
        while len(self.buffer) <= self.batch_size:
            if self.collect_once:
                self.sampling_data()
            else:
                rec.wait_for(rec.inserted + 1)
        try:
            while True:
                if not self.collect_once:
                    rec.poll(self.polls_per_step)
                self.learn_step()
                t = self.learn_idx
                if t % self.target_update_interval == 0:
                    print("Updating Target Network..")
                    self.tgt_model.load_state_dict(self.model.state_dict())
                if t % self.save_interval == 0:
                    print("Saving Model..")
                    self.save_model(t)
                if t % self.publish_param_interval == 0:
                    rec.set_worker_weights(self.model)
                if t >= self.max_step:
                    self.save_model(t)
                    break
        finally:
            rec.cleanup()
            self.writer.flush()
        return self.last

    def model_path(self, idx):
        return os.path.join(self.save_dir, f"model{idx}.pth")

    def save_model(self, idx):
        path = save_model(self.model, self.model_path(idx))
        save_train_state(path, target=self.tgt_model, optimizers=[self.optimizer], schedulers=[self.scheduler],
                         counters={"learn_idx": self.learn_idx})
        return path

    def load_model(self, idx):
        print(f"loading weights_{idx}")
        load_model(self.model, self.model_path(idx))


def main(argv=None):
    p = argparse.ArgumentParser(description="Single-node Ape-X (ApeX.py)")
    p.add_argument("--env", default="MountainCar-v0")
    p.add_argument("--n-workers", type=int, default=20)
    p.add_argument("--max-step", type=float, default=1e5)
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--save-dir", default=".")
    p.add_argument("--collect-once", action="store_true", help="reference behaviour: collect once, train offline")
    a = p.parse_args(argv)
    t = train_DQN(a.env, seed=a.seed, n_workers=a.n_workers, max_step=a.max_step, batch_size=a.batch_size,
                  save_dir=a.save_dir, collect_once=a.collect_once)
    print(t.train())


if __name__ == "__main__":
    main()
