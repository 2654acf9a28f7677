"""Amortized Q-learning trainers (reference AQL.py:17-182 and AQL_dis.py:18-170;
SURVEY R11, R12, §3.5).

One learner update (``aql_update``), shared by both trainers:

1. sample (s, a, r, s', d, a_mu, w, idx) from the AQL PER buffer;
2. proposal loss ``-log pi(a*_Q | s) - ent_lam * H(pi(.|s))`` where ``a*_Q`` is the
   candidate with the highest online Q; Adam step on the proposal, clip 40;
3. (AQL_dis) hard-copy proposal -> target proposal every step;
4. ``compute_loss_AQL`` (n-step double-Q Huber over the candidate set, the s_t
   candidates re-used for s'), Adam step on the critic, clip 40, priorities written
   back *before* the optimizer step (reference ordering);
5. (AQL_dis) ``reset_noise`` on the online and target NoisyNets.

``train_AQL`` = AQL.py (single process, Pendulum, lr 1e-4 with cosine annealing, beta
annealed over ``max_step``, behaviour epsilon 0.5 w.p. .9 else 0.05).
``train_AQL_dis`` = AQL_dis.py (BatchRecorder of CPU AQL workers, weights broadcast
every outer iteration, ``total_ep_len // batch`` SGD steps per iteration, target sync
every 20 iterations, checkpoint every 200).
"""
from __future__ import annotations

import argparse
import math
import os
import random

import numpy as np
import torch

from .. import envs
from ..algo.losses import compute_loss_AQL
from ..models.aql import AQL
from ..replay.buffers import CustomPrioritizedReplayBuffer_AQL
from ..utils import set_global_seeds
from ..utils.checkpoint import load_model, save_model, save_train_state
from ..utils.tb import SummaryWriter


def sample_aql_batch(buffer, batch_size, beta, device):
    s, a, r, s2, d, a_mu, w, idx = buffer.sample(batch_size, beta)
    f32 = lambda x: torch.as_tensor(np.asarray(x, dtype=np.float32), device=device)  # noqa: E731
    batch = (f32(s), torch.as_tensor(np.asarray(a), dtype=torch.int64, device=device), f32(r), f32(s2), f32(d),
             f32(a_mu), f32(w))
    return batch, idx


def aql_update(model, target_model, buffer, optimizer_q, optimizer_proposal, batch_size, beta, gamma, n_steps,
               ent_lam, device, copy_proposal_to_target=False, reset_noise=False, max_norm=40.0, fused=None):
    batch = sample_aql_batch(buffer, batch_size, beta, device)
    (state, action, reward, next_state, done, a_mu, weights), indices = batch
    # proposal loss: imitate the critic's best candidate, entropy bonus
    q_values = model(state, a_mu)
    embed_state = model.q.embedding_feature(state)
    dist = model.proposal.evaluate(embed_state)
    # reshape(B, -1) as in AQL.py:86: for a discrete proposal the [B, 1] value broadcasts
    # against the Categorical's [B] batch into a [B, B] log-prob matrix (reference quirk, kept)
    best = a_mu[torch.arange(batch_size, device=a_mu.device), q_values.max(1)[1]].reshape(batch_size, -1)
    loss_p = torch.mean(-dist.log_prob(best) - ent_lam * dist.entropy())
    optimizer_proposal.zero_grad()
    loss_p.backward()
    torch.nn.utils.clip_grad_norm_(model.proposal.parameters(), max_norm)
    optimizer_proposal.step()
    if copy_proposal_to_target:
        target_model.proposal.load_state_dict(model.proposal.state_dict())
    # critic loss
    batch_t = (state, action, reward, next_state, done, a_mu, weights)
    if fused is not None:  # (FusedAQL online, FusedAQL target): no-grad s' critics on the HIP kernel
        loss_q, prios = compute_loss_AQL_fused(model, target_model, fused[0], fused[1], batch_t, n_steps, gamma)
    else:
        loss_q, prios = compute_loss_AQL(model, target_model, batch_t, n_steps=n_steps, gamma=gamma)
    optimizer_q.zero_grad()
    loss_q.backward()
    torch.nn.utils.clip_grad_norm_(model.q.parameters(), max_norm)
    buffer.update_priorities(indices, prios)
    optimizer_q.step()
    if reset_noise:
        model.reset_noise()
        target_model.reset_noise()
    return loss_q, loss_p


def compute_loss_AQL_fused(model, target_model, fused, fused_tgt, batch, n_steps, gamma=0.99):
    """``compute_loss_AQL`` with the two no-grad critic evaluations at s' (online and
    target, utils.py:48-49) on the fused HIP kernel; Q(s, a_mu) keeps autograd."""
    from ..algo.losses import _td_terms, huber_weighted, priorities_from_td

    states, actions, rewards, next_states, dones, a_mu, weights = batch
    q_values = model(states, a_mu)
    with torch.no_grad():
        next_q = fused.candidate_q(next_states, a_mu)
        tgt_next_q = fused_tgt.candidate_q(next_states, a_mu)
    td = _td_terms(q_values, next_q, tgt_next_q, actions, rewards, dones, n_steps, gamma)
    return huber_weighted(td, weights), priorities_from_td(td).detach().cpu().numpy()


class VectorAQLActors:
    """GPU-batched AQL acting for ``n_envs`` host envs: one proposal + candidate-Q +
    epsilon-greedy launch sequence per env step for all envs (FusedAQL), instead of one
    CPU process and ~20 small ops + ``.cpu()`` per env per step (batchrecoder_AQL.py).
    Same recording contract as ``BatchRecorder.record_batch``: every env plays one
    episode, raw (s, a, r, s', d, a_mu) transitions go into the buffer."""

    def __init__(self, env_id, n_envs, buffer, model, seed=0, max_episode_length=50000, writer=None,
                 eps_base=0.4, eps_alpha=7.0):
        from ..algo.schedules import actor_epsilon
        from ..models.aql_fused import FusedAQL

        self.envs = [envs.make(env_id) for _ in range(n_envs)]
        for i, e in enumerate(self.envs):
            e.seed(seed + i)
        self.buffer = buffer
        self.model = model
        self.fused = FusedAQL(model, seed=seed)
        self.max_episode_length = int(max_episode_length)
        self.writer = writer
        self.episode_idx = 0
        eps = actor_epsilon(np.arange(n_envs), n_envs, eps_base, eps_alpha)
        self.eps = torch.as_tensor(np.atleast_1d(eps), dtype=torch.float32, device=self.fused.device)

    def record_batch(self) -> int:
        E = len(self.envs)
        states = [e.reset() for e in self.envs]
        active = np.ones(E, dtype=bool)
        ep_r, ep_len = np.zeros(E), np.zeros(E, dtype=np.int64)
        while active.any():
            ids = np.nonzero(active)[0]
            st = np.stack([np.asarray(states[i], dtype=np.float32) for i in ids])
            with torch.no_grad():
                idx, am, act = self.fused.act(st, self.eps[torch.as_tensor(ids, device=self.eps.device)])
            idx, am, act = idx.cpu().numpy(), am.cpu().numpy(), act.cpu().numpy()
            for j, i in enumerate(ids):
                a_env = act[j] if self.fused.cont else int(act[j])
                s2, r, d, _ = self.envs[i].step(a_env)
                a_mu = am[j] if self.fused.cont else am[j].astype(np.int64)
                self.buffer.add(states[i], int(idx[j]), r, s2, d, a_mu)
                states[i] = s2
                ep_r[i] += r
                ep_len[i] += 1
                if d or ep_len[i] >= self.max_episode_length:
                    active[i] = False
                    if self.writer is not None:
                        self.writer.add_scalar("actor/episode_reward", float(ep_r[i]), self.episode_idx)
                        self.writer.add_scalar("actor/episode_length", int(ep_len[i]), self.episode_idx)
                    self.episode_idx += 1
        return int(ep_len.sum())

    def set_worker_weights(self, model) -> None:
        if model is not self.model:
            self.model.load_state_dict(model.state_dict())

    def cleanup(self) -> None:
        for e in self.envs:
            e.close()


class _AQLBase:
    def _build(self, env_id, propose_sample, uniform_sample, action_var, device, buffer_size, prior_alpha, lr, seed,
               writer):
        if seed is not None:
            set_global_seeds(seed, use_torch=True)
        self.device = torch.device(device)
        self.env = envs.make(env_id)
        if seed is not None:
            self.env.seed(seed)
        kw = dict(propose_sample=propose_sample, uniform_sample=uniform_sample, action_var=action_var,
                  device=self.device)
        self.model = AQL(env=self.env, **kw).to(self.device)
        self.target_model = AQL(env=self.env, **kw).to(self.device)
        self.target_model.load_state_dict(self.model.state_dict())
        self.replay_buffer = CustomPrioritizedReplayBuffer_AQL(int(buffer_size), alpha=prior_alpha)
        self.lr = lr
        self.optimizer_q = torch.optim.Adam(self.model.q.parameters(), lr)
        self.optimizer_proposal = torch.optim.Adam(self.model.proposal.parameters(), lr)
        self.writer = writer if writer is not None else SummaryWriter(comment=f"-{self.env.unwrapped.spec.id}-learner")

    @staticmethod
    def update_target(current_model, target_model):
        target_model.load_state_dict(current_model.state_dict())

    def model_path(self, idx):
        return os.path.join(self.save_dir, f"model{idx}.pth")

    def save_model(self, idx):
        path = save_model(self.model, self.model_path(idx))
        save_train_state(path, target=self.target_model, optimizers=[self.optimizer_q, self.optimizer_proposal],
                         schedulers=[self.scheduler_q, self.scheduler_proposal], counters={"idx": idx})
        return path

    def load_model(self, idx):
        print(f"loading weights_{idx}")
        load_model(self.model, self.model_path(idx))


class train_AQL(_AQLBase):  # AQL.py train_DQN
    def __init__(self, env_id, max_step=1e6, prior_alpha=0.6, prior_beta_start=0.4, epsilon_start=1,
                 epsilon_final=0.01, epsilon_decay=1e4, batch_size=32, gamma=0.99, target_update_interval=1000,
                 save_interval=1e4, propose_sample=100, uniform_sample=100, action_var=0.25, ent_lam=0.8, lr=1e-4,
                 device=None, seed=None, save_dir=".", writer=None, buffer_size=100_000):
        self.prior_beta_start = prior_beta_start
        self.max_step = int(max_step)
        self.batch_size = int(batch_size)
        self.gamma = gamma
        self.target_update_interval = int(target_update_interval)
        self.save_interval = int(save_interval)
        self.ent_lam = ent_lam
        self.save_dir = save_dir
        # unused by the reference loop (it uses the 0.5 / 0.05 behaviour epsilon), kept for the API
        self.epsilon_by_frame = lambda t: epsilon_final + (epsilon_start - epsilon_final) * math.exp(-t / epsilon_decay)
        device = device if device is not None else ("cuda:0" if torch.cuda.is_available() else "cpu")
        self._build(env_id, propose_sample, uniform_sample, action_var, device, buffer_size, prior_alpha, lr, seed,
                    writer)
        self.fused = None
        if self.device.type == "cuda":  # no-grad s' critics on the fused HIP kernel
            from ..models.aql_fused import FusedAQL

            self.fused = (FusedAQL(self.model), FusedAQL(self.target_model))
        self.scheduler_q = torch.optim.lr_scheduler.CosineAnnealingLR(self.optimizer_q, T_max=self.max_step,
                                                                      eta_min=lr / 1000)
        self.scheduler_proposal = torch.optim.lr_scheduler.CosineAnnealingLR(self.optimizer_proposal,
                                                                             T_max=self.max_step, eta_min=lr / 1000)
        self.episode_rewards: list[float] = []

    def beta_by_frame(self, t):
        return min(1.0, self.prior_beta_start + t * (1.0 - self.prior_beta_start) / self.max_step)

    def compute_td_loss(self, batch_size, beta):
        loss_q, loss_p = aql_update(self.model, self.target_model, self.replay_buffer, self.optimizer_q,
                                    self.optimizer_proposal, batch_size, beta, self.gamma, 1, self.ent_lam,
                                    self.device, fused=self.fused)
        self.scheduler_proposal.step()
        self.scheduler_q.step()
        return loss_q, loss_p

    def train(self):
        ep_r, ep_idx, ep_len = 0.0, 0, 0
        state = self.env.reset()
        for frame_idx in range(self.max_step):
            epsilon = 0.5 if random.random() > 0.1 else 0.05
            action, a_mu, _ = self.model.act(state, epsilon)
            a_mu = a_mu[0]
            next_state, reward, done, _ = self.env.step(a_mu[action])
            self.replay_buffer.add(state, action, reward, next_state, done, a_mu)
            state = next_state
            ep_r += reward
            ep_len += 1
            if done:
                state = self.env.reset()
                self.episode_rewards.append(ep_r)
                self.writer.add_scalar("actor/episode_reward", ep_r, ep_idx)
                self.writer.add_scalar("actor/episode_length", ep_len, ep_idx)
                ep_r, ep_len = 0.0, 0
                ep_idx += 1
            if len(self.replay_buffer) > self.batch_size:
                loss_q, loss_p = self.compute_td_loss(self.batch_size, self.beta_by_frame(frame_idx))
                self.writer.add_scalar("learner/loss_q", float(loss_q.detach()), frame_idx)
                self.writer.add_scalar("learner/loss_proposal", float(loss_p.detach()), frame_idx)
            if frame_idx % self.target_update_interval == 0:
                self.update_target(self.model, self.target_model)
            if frame_idx % self.save_interval == 0 or frame_idx == self.max_step - 1:
                self.save_model(frame_idx)
        self.env.close()
        self.writer.flush()
        return self.episode_rewards


class train_AQL_dis(_AQLBase):  # AQL_dis.py train_DQN
    def __init__(self, env_id, max_step=1e6, prior_alpha=0.6, prior_beta_start=0.4, publish_param_interval=5,
                 device=None, n_steps=1, batch_size=32, gamma=0.99, target_update_interval=20, save_interval=200,
                 propose_sample=1, uniform_sample=50, action_var=0.25, ent_lam=0.8, n_workers=10, lr=1e-3, seed=0,
                 save_dir=".", writer=None, buffer_size=1e7, start_method="spawn", aql_dup_by_obs_dim=False,
                 max_episode_length=50000, gpu_actors: int = 0, fused: bool | None = None):
        from .batchrecorder import KIND_AQL, BatchRecorder

        self.prior_beta_start = prior_beta_start
        self.max_step = int(max_step)
        self.batch_size = int(batch_size)
        self.gamma = gamma
        self.target_update_interval = int(target_update_interval)
        self.publish_param_interval = publish_param_interval  # unused by the reference loop too
        self.save_interval = int(save_interval)
        self.ent_lam = ent_lam
        self.n_workers = int(n_workers)
        self.n_steps = int(n_steps)
        self.save_dir = save_dir
        device = device if device is not None else ("cuda:0" if torch.cuda.is_available() else "cpu")
        self._build(env_id, propose_sample, uniform_sample, action_var, device, buffer_size, prior_alpha, lr, seed,
                    writer)
        self.scheduler_q = torch.optim.lr_scheduler.StepLR(self.optimizer_q, step_size=100, gamma=0.99)
        self.scheduler_proposal = torch.optim.lr_scheduler.StepLR(self.optimizer_proposal, step_size=100, gamma=0.99)
        use_fused = (self.device.type == "cuda") if fused is None else fused
        self.fused = None
        if use_fused:
            from ..models.aql_fused import FusedAQL

            self.fused = (FusedAQL(self.model), FusedAQL(self.target_model))
        if gpu_actors:
            actor_model = AQL(env=self.env, propose_sample=propose_sample, uniform_sample=uniform_sample,
                              action_var=action_var, device=self.device).to(self.device)
            self.recoder = VectorAQLActors(env_id, gpu_actors, self.replay_buffer, actor_model, seed=0,
                                           max_episode_length=max_episode_length, writer=self.writer)
            self.learn_idx = 0
            return
        cpu_model = AQL(env=self.env, propose_sample=propose_sample, uniform_sample=uniform_sample,
                        action_var=action_var, device="cpu")
        self.recoder = BatchRecorder(env_id, env_seed=0, n_workers=self.n_workers, buffer=self.replay_buffer,
                                     max_episode_length=max_episode_length, writer=self.writer, kind=KIND_AQL,
                                     start_method=start_method, aql_dup_by_obs_dim=aql_dup_by_obs_dim,
                                     aql_kwargs=dict(propose_sample=propose_sample, uniform_sample=uniform_sample,
                                                     action_var=action_var),
                                     model=cpu_model)
        self.learn_idx = 0

    def beta_by_frame(self, t):
        # AQL_dis.py:59 (operator precedence kept: .../max_step*n_workers)
        return min(1.0, self.prior_beta_start + t * (1.0 - self.prior_beta_start) / self.max_step * self.n_workers)

    def compute_td_loss(self, batch_size, beta):
        return aql_update(self.model, self.target_model, self.replay_buffer, self.optimizer_q, self.optimizer_proposal,
                          batch_size, beta, self.gamma, self.n_steps, self.ent_lam, self.device,
                          copy_proposal_to_target=True, reset_noise=True, fused=self.fused)

    def train(self):
        try:
            for frame_idx in range(self.max_step):
                self.model.q.train()
                self.target_model.q.train()
                self.recoder.set_worker_weights(self.model)
                total_ep = self.recoder.record_batch()
                for _ in range(total_ep // self.batch_size):
                    if len(self.replay_buffer) > self.batch_size:
                        loss_q, loss_p = self.compute_td_loss(self.batch_size, self.beta_by_frame(frame_idx))
                        self.writer.add_scalar("learner/loss_q", float(loss_q.detach()), self.learn_idx)
                        self.writer.add_scalar("learner/loss_proposal", float(loss_p.detach()), self.learn_idx)
                    self.learn_idx += 1
                if frame_idx % self.target_update_interval == 0:
                    self.update_target(self.model, self.target_model)
                if frame_idx % self.save_interval == 0 or frame_idx == self.max_step - 1:
                    self.save_model(frame_idx)
        finally:
            self.recoder.cleanup()
            self.writer.flush()
        return getattr(self.recoder, "episodes", self.recoder.episode_idx)


def main(argv=None):
    p = argparse.ArgumentParser(description="AQL trainers (AQL.py / AQL_dis.py)")
    p.add_argument("--dis", action="store_true", help="multi-worker AQL_dis trainer")
    p.add_argument("--env", default=None)
    p.add_argument("--max-step", type=float, default=None)
    p.add_argument("--n-workers", type=int, default=10)
    p.add_argument("--save-dir", default=".")
    a = p.parse_args(argv)
    if a.dis:
        t = train_AQL_dis(a.env or "CartPole-v0", max_step=a.max_step or 1e6, n_workers=a.n_workers,
                          save_dir=a.save_dir)
    else:
        t = train_AQL(a.env or "Pendulum-v0", max_step=a.max_step or 1e6, save_dir=a.save_dir)
    t.train()


if __name__ == "__main__":
    main()
