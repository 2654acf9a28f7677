"""Single-process prioritized double-DQN trainer (reference DQN.py:15-149).

BASELINE config 1: CartPole on CPU.  Semantics kept from the reference:

* PER(1e5, alpha .6) with max-priority inserts, beta annealed 0.4 -> 1 over 1000 frames
* epsilon(t) = 0.01 + 0.99 exp(-t/500); one gradient step per env step once
  ``len(replay) > batch_size``
* n = 1 double-DQN Huber loss (``compute_loss``), Adam(lr 1e-3) + StepLR(1000, .99),
  no gradient clipping
* SURVEY Q9 ordering: ``scheduler.step()`` and ``update_priorities`` happen *before*
  ``optimizer.step()``
* target sync every ``target_update_interval`` frames including frame 0; checkpoints
  ``model{t}.pth`` every ``save_interval`` frames and at the last frame

``python -m apex_amd.trainers.dqn --env CartPole-v0 --max-step 100000`` (or
``--eval N`` to play a saved checkpoint greedily, the reference's ``training=False``).
"""
from __future__ import annotations

import argparse
import os

import numpy as np
import torch

from .. import envs
from ..algo.losses import compute_loss
from ..algo.schedules import beta_by_frame, epsilon_by_frame, step_scheduler_early
from ..models.dqn import DuelingDQN
from ..replay.buffers import PrioritizedReplayBuffer
from ..utils import set_global_seeds
from ..utils.checkpoint import load_model, save_model, save_train_state
from ..utils.tb import SummaryWriter


class train_DQN:  # noqa: N801  (reference class name)
    def __init__(self, env_id, max_step=1e5, prior_alpha=0.6, prior_beta_start=0.4, epsilon_start=1.0,
                 epsilon_final=0.01, epsilon_decay=500, batch_size=32, gamma=0.99, target_update_interval=1000,
                 save_interval=1e4, lr=1e-3, buffer_size=100_000, device=None, seed=None, save_dir=".",
                 writer=None, exact_mass=False, log_every=1):
        self.prior_beta_start = prior_beta_start
        self.max_step = int(max_step)
        self.batch_size = int(batch_size)
        self.gamma = gamma
        self.target_update_interval = int(target_update_interval)
        self.save_interval = int(save_interval)
        self.eps = (float(epsilon_start), float(epsilon_final), float(epsilon_decay))
        self.save_dir = save_dir
        self.log_every = max(1, int(log_every))
        if seed is not None:
            set_global_seeds(seed, use_torch=True)
        self.device = torch.device(device if device is not None else ("cuda:0" if torch.cuda.is_available() else "cpu"))
        self.env = envs.make(env_id)
        if seed is not None:
            self.env.seed(seed)
        self.model = DuelingDQN(self.env).to(self.device)
        self.target_model = DuelingDQN(self.env).to(self.device)
        self.target_model.load_state_dict(self.model.state_dict())
        self.replay_buffer = PrioritizedReplayBuffer(buffer_size, alpha=prior_alpha, exact_mass=exact_mass)
        self.optimizer = torch.optim.Adam(self.model.parameters(), lr=lr)
        self.scheduler = torch.optim.lr_scheduler.StepLR(self.optimizer, step_size=1000, gamma=0.99)
        self.writer = writer if writer is not None else SummaryWriter(comment=f"-{self.env.unwrapped.spec.id}-learner")
        self.episode_rewards: list[float] = []
        self.losses: list[float] = []

    def beta_by_frame(self, frame_idx):
        return beta_by_frame(frame_idx, self.prior_beta_start, 1000.0)

    def epsilon_by_frame(self, frame_idx):
        return epsilon_by_frame(frame_idx, *self.eps)

    @staticmethod
    def update_target(current_model, target_model):
        target_model.load_state_dict(current_model.state_dict())

    def compute_td_loss(self, batch_size, beta):
        s, a, r, s2, d, w, idx = self.replay_buffer.sample(batch_size, beta)
        dev = self.device
        batch = (torch.as_tensor(np.asarray(s), dtype=torch.float32, device=dev),
                 torch.as_tensor(np.asarray(a), dtype=torch.int64, device=dev),
                 torch.as_tensor(np.asarray(r), dtype=torch.float32, device=dev),
                 torch.as_tensor(np.asarray(s2), dtype=torch.float32, device=dev),
                 torch.as_tensor(np.asarray(d), dtype=torch.float32, device=dev),
                 torch.as_tensor(np.asarray(w), dtype=torch.float32, device=dev))
        loss, prios = compute_loss(self.model, self.target_model, batch, 1, self.gamma)
        self.optimizer.zero_grad()
        loss.backward()
        step_scheduler_early(self.scheduler)               # Q9: LR decays one step early
        self.replay_buffer.update_priorities(idx, prios)   # Q9: before optimizer.step
        self.optimizer.step()
        return loss

    def train(self):
        episode_reward, episode_idx, episode_length = 0.0, 0, 0
        state = self.env.reset()
        for frame_idx in range(self.max_step):
            epsilon = self.epsilon_by_frame(frame_idx)
            action, _ = self.model.act(torch.as_tensor(np.asarray(state), dtype=torch.float32, device=self.device),
                                       epsilon)
            next_state, reward, done, _ = self.env.step(action)
            self.replay_buffer.add(state, action, reward, next_state, done)
            state = next_state
            episode_reward += reward
            episode_length += 1
            if done:
                state = self.env.reset()
                self.episode_rewards.append(episode_reward)
                self.writer.add_scalar("actor/episode_reward", episode_reward, episode_idx)
                self.writer.add_scalar("actor/episode_length", episode_length, episode_idx)
                episode_reward, episode_length = 0.0, 0
                episode_idx += 1
            if len(self.replay_buffer) > self.batch_size:
                loss = self.compute_td_loss(self.batch_size, self.beta_by_frame(frame_idx))
                if frame_idx % self.log_every == 0:
                    lv = float(loss.detach())
                    self.losses.append(lv)
                    self.writer.add_scalar("learner/loss", lv, frame_idx)
            if frame_idx % self.target_update_interval == 0:
                print("update target...")
                self.update_target(self.model, self.target_model)
            if frame_idx % self.save_interval == 0 or frame_idx == self.max_step - 1:
                print("save model...")
                self.save_model(frame_idx)
        self.writer.flush()
        return self.episode_rewards

    def model_path(self, idx) -> str:
        return os.path.join(self.save_dir, f"model{idx}.pth")

    def save_model(self, idx):
        path = save_model(self.model, self.model_path(idx))
        save_train_state(path, target=self.target_model, optimizers=[self.optimizer], schedulers=[self.scheduler],
                         counters={"frame_idx": idx})
        return path

    def load_model(self, idx):
        print(f"loading weights_{idx}")
        load_model(self.model, self.model_path(idx))

    def evaluate(self, n_episodes=10, render=False):
        """Greedy play (the reference's ``training=False`` branch)."""
        returns = []
        for _ in range(n_episodes):
            s, er = self.env.reset(), 0.0
            while True:
                if render:
                    self.env.render()
                a, _ = self.model.act(torch.as_tensor(np.asarray(s), dtype=torch.float32, device=self.device), 0)
                s, r, d, _ = self.env.step(a)
                er += r
                if d:
                    returns.append(er)
                    break
        return returns


def main(argv=None):
    p = argparse.ArgumentParser(description="Prioritized double-DQN (DQN.py)")
    p.add_argument("--env", default="CartPole-v0")
    p.add_argument("--max-step", type=float, default=1e5)
    p.add_argument("--batch-size", type=int, default=32)
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--save-dir", default=".")
    p.add_argument("--device", default=None)
    p.add_argument("--eval", type=int, default=None, metavar="IDX", help="load model{IDX}.pth and play greedily")
    p.add_argument("--render", action="store_true")
    a = p.parse_args(argv)
    t = train_DQN(a.env, max_step=a.max_step, batch_size=a.batch_size, seed=a.seed, save_dir=a.save_dir,
                  device=a.device)
    if a.eval is None:
        t.train()
    else:
        t.device = torch.device("cpu")
        t.model.to("cpu")
        t.load_model(a.eval)
        for r in t.evaluate(10, a.render):
            print(r)
    t.env.close()


if __name__ == "__main__":
    main()
