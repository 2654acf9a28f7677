"""Amortized Q-Learning model: NoisyNet critic over proposed action candidates
(reference model.py:169-390).

* ``Q_Network``: state trunk ``features`` (Linear(obs->128)+ReLU), ``q_feature``
  (Linear(obs->64)-ReLU-Linear(64->64)-ReLU), candidate encoder ``action_out``
  (continuous: Linear(A->128)-ReLU-Linear(128->64)-ReLU; discrete:
  Linear(1->64)-ReLU) and a NoisyLinear head 128->64->1 giving one Q per
  (state, candidate).
* ``Proposal_Network``: ``dist_feature`` Linear(128->128)-ReLU-Linear(128->A) on the
  critic's state embedding; samples ``propose_sample`` candidates from
  MVN(mu, diag(action_var)) / Categorical(logits) plus ``uniform_sample`` uniform
  candidates (uniform over the Box, or without replacement over discrete actions).
* ``AQL``: T = propose + uniform candidates (uniform clamped to n for discrete).

Kept behaviours (documented quirks): ``forward`` also runs the epsilon-greedy argmax
(the reference returns ``q.act(...)[1]``), greedy action taken from row 0 only, and
the critic's image path is unsupported (the reference fails on 3-D observations with
a reshape error; here a ValueError says so).  The hot path for the distributed AQL
engine batches the [B, T] candidate MLP on the GPU (see ``apex_amd.engine.aql``).
"""
from __future__ import annotations

import random

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Categorical, MultivariateNormal, Uniform

from ..envs.spaces import is_box
from .dqn import init
from .noisy import NoisyLinear


class Q_Network(nn.Module):
    A_OUT = 64
    F_OUT = 64

    def __init__(self, input_shape, num_actions, total_sample, env_iscontinuous, device=None):
        super().__init__()
        self.device = device
        self.input_shape = tuple(input_shape)
        if len(self.input_shape) == 3:
            raise ValueError("AQL critic supports vector observations only (reference model.py:286-288 reshapes "
                             "the trunk output to (-1, 128), which fails for the Nature-CNN trunk)")
        self.cnn = False
        self.total_sample = total_sample
        self.num_actions = num_actions
        self.env_iscontinuous = env_iscontinuous
        self.a_out_unit = self.A_OUT
        self.feature_out_unit = self.F_OUT
        self.concat_unit = self.A_OUT + self.F_OUT
        obs = self.input_shape[0]
        self.features = nn.Sequential(init(nn.Linear(obs, 128)), nn.ReLU())
        self.q_feature = nn.Sequential(init(nn.Linear(obs, 64)), nn.ReLU(), init(nn.Linear(64, self.F_OUT)), nn.ReLU())
        if env_iscontinuous:
            self.action_out = nn.Sequential(nn.Linear(num_actions, 128), nn.ReLU(), nn.Linear(128, self.A_OUT), nn.ReLU())
        else:
            self.action_out = nn.Sequential(nn.Linear(1, self.A_OUT), nn.ReLU())
        self.advantage1 = NoisyLinear(self.concat_unit, 64, device=device)
        self.advantage2 = NoisyLinear(64, 1, device=device)

    def forward(self, x, q_f=None):
        x = x.reshape(-1, self.concat_unit)
        return self.advantage2(F.relu(self.advantage1(x)))

    def embedding_feature(self, x):
        return self.features(x).reshape(-1, 128)

    def reset_noise(self):
        self.advantage1.reset_noise()
        self.advantage2.reset_noise()

    def candidate_q(self, state, a_mu):
        """Q[B, T] for every (state, candidate) pair, no action selection."""
        T = self.total_sample
        if self.env_iscontinuous:
            a_mu = a_mu.reshape(-1, T, self.num_actions)
            a_out = self.action_out(a_mu.reshape(-1, self.num_actions)).reshape(-1, T, self.A_OUT)
        else:
            a_out = self.action_out(a_mu.reshape(-1, 1).float()).reshape(-1, T, self.A_OUT)
        q_f = self.q_feature(state).repeat(1, T).reshape(-1, T, self.F_OUT)
        x = F.relu(torch.cat([a_out, q_f], dim=2))
        return self.forward(x).reshape(a_mu.shape[0], T)

    def act(self, state, a_mu, epsilon):
        q_values = self.candidate_q(state, a_mu)
        if random.random() > epsilon:
            action = torch.argmax(q_values, dim=1)[0].cpu().numpy()
        else:
            action = random.choice(list(range(self.total_sample)))
        return action, q_values


class Proposal_Network(nn.Module):
    def __init__(self, env, propose_sample=100, uniform_sample=100, action_var=0.25, device=None):
        super().__init__()
        self.device = device
        self.env = env
        self.input_shape = env.observation_space.shape
        self.env_iscontinuous = is_box(env.action_space)
        self.uniform_sample = uniform_sample
        self.propose_sample = propose_sample
        self.num_actions = env.action_space.shape[0] if self.env_iscontinuous else env.action_space.n
        self.dist_feature = nn.Sequential(init(nn.Linear(128, 128)), nn.ReLU(), init(nn.Linear(128, self.num_actions)))
        # a plain tensor, deliberately not a buffer: not part of the state_dict (model.py:357)
        self.action_var = torch.full((self.num_actions,), float(action_var))
        if self.env_iscontinuous:
            self.uniform = Uniform(torch.as_tensor(env.action_space.low, dtype=torch.float32),
                                   torch.as_tensor(env.action_space.high, dtype=torch.float32))

    def _dev(self, t):
        return t.to(self.device) if self.device is not None else t

    def forward(self, embed_state):
        mu = self._dev(self.dist_feature(embed_state))
        if self.env_iscontinuous:
            dist = MultivariateNormal(mu, self._dev(torch.diag(self.action_var)))
            a_uniform = self._dev(self.uniform.sample([mu.shape[0], self.uniform_sample]))
            a_dist = dist.sample([self.propose_sample]).reshape((-1, self.propose_sample, self.num_actions))
            return torch.cat([a_uniform, a_dist], dim=1)
        dist = Categorical(logits=mu)
        a_dist = dist.sample([self.propose_sample]).reshape(mu.shape[0], self.propose_sample)
        a_uniform = np.random.choice(torch.arange(self.num_actions), size=self.uniform_sample, replace=False)
        a_uniform = self._dev(torch.LongTensor(a_uniform).reshape(mu.shape[0], self.uniform_sample))
        return torch.cat([a_uniform, a_dist], dim=1)

    def evaluate(self, embed_state):
        mu = self.dist_feature(embed_state)
        if self.env_iscontinuous:
            return MultivariateNormal(mu, self._dev(torch.diag(self.action_var)))
        return Categorical(logits=mu)


class AQL(nn.Module):
    def __init__(self, env, propose_sample=100, uniform_sample=400, action_var=0.25, device="cuda"):
        super().__init__()
        self.device = device
        self.env = env
        self.input_shape = env.observation_space.shape
        self.env_iscontinuous = is_box(env.action_space)
        if self.env_iscontinuous:
            self.num_actions = env.action_space.shape[0]
            self.uniform_sample = uniform_sample
        else:
            self.num_actions = env.action_space.n
            self.uniform_sample = min(uniform_sample, env.action_space.n)
        self.propose_sample = propose_sample
        self.total_sample = propose_sample + self.uniform_sample
        self.q = Q_Network(self.input_shape, self.num_actions, self.total_sample, self.env_iscontinuous, device)
        self.proposal = Proposal_Network(env, propose_sample, self.uniform_sample, action_var, device)

    def forward(self, state, a_mu):
        _, q_values = self.q.act(state, a_mu, 0)
        return q_values

    def act(self, state, epsilon):
        with torch.no_grad():
            state = torch.FloatTensor(np.asarray(state)).to(self.device)
            x = self.q.embedding_feature(state)
            a_mu = self.proposal.forward(x)
            action, q_values = self.q.act(state, a_mu, epsilon)
            return action, a_mu.cpu().numpy(), q_values

    def reset_noise(self):
        self.q.reset_noise()
