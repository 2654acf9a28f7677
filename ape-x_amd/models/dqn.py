"""Dueling Q-network (reference model.py:14-107).

Architecture and checkpoint contract:

* 3-D observations -> Nature CNN trunk ``features.{0,2,4}`` =
  Conv(C->32,k8,s4) / Conv(32->64,k4,s2) / Conv(64->64,k3,s1), ReLU after each;
  otherwise ``features.0`` = Linear(obs->128) + ReLU.
* Two heads with **128** hidden units: ``advantage.{0,2}`` and ``value.{0,2}``.
* ``Q = V + A - mean_a(A)``.
* Orthogonal init with ReLU gain, zero bias.

The state_dict (keys, shapes, fp32) is byte-compatible with the reference so a
``torch.save(model.state_dict())`` from either side loads into the other.  The
module is also the parameter container of the HIP learner: ``flatten_parameters``
re-seats every parameter as a view of one contiguous fp32 buffer, so the fused
optimizer / grad-norm kernels and the single RCCL all-reduce / broadcast operate on
one 3.5 MB allocation while ``state_dict()`` keeps the reference layout.
"""
from __future__ import annotations

import random
from types import SimpleNamespace

import numpy as np
import torch
import torch.nn as nn

from ..envs.spaces import Box, Discrete


class Flatten(nn.Module):
    def forward(self, x):
        return x.view(x.size(0), -1)


def init_(module, weight_init, bias_init, gain=1.0):
    weight_init(module.weight.data, gain=gain)
    bias_init(module.bias.data)
    return module


def init(module):
    """Orthogonal(relu gain) weights, zero bias (model.py:97-107)."""
    return init_(module, nn.init.orthogonal_, lambda b: nn.init.constant_(b, 0), nn.init.calculate_gain("relu"))


def env_spec(obs_shape, n_actions: int):
    """A stand-in ``env`` carrying only the spaces, for building models without an env."""
    return SimpleNamespace(observation_space=Box(0, 255, shape=tuple(obs_shape), dtype=np.uint8),
                           action_space=Discrete(n_actions))


class DuelingDQN(nn.Module):
    HIDDEN = 128

    def __init__(self, env):
        super().__init__()
        self.input_shape = tuple(env.observation_space.shape)
        self.cnn = len(self.input_shape) == 3
        self.num_actions = int(env.action_space.n)
        self.flatten = Flatten()
        if self.cnn:
            c = self.input_shape[0]
            self.features = nn.Sequential(
                init(nn.Conv2d(c, 32, kernel_size=8, stride=4)), nn.ReLU(),
                init(nn.Conv2d(32, 64, kernel_size=4, stride=2)), nn.ReLU(),
                init(nn.Conv2d(64, 64, kernel_size=3, stride=1)), nn.ReLU(),
            )
        else:
            self.features = nn.Sequential(init(nn.Linear(self.input_shape[0], self.HIDDEN)), nn.ReLU())
        f = self._feature_size()
        self.advantage = nn.Sequential(init(nn.Linear(f, self.HIDDEN)), nn.ReLU(),
                                       init(nn.Linear(self.HIDDEN, self.num_actions)))
        self.value = nn.Sequential(init(nn.Linear(f, self.HIDDEN)), nn.ReLU(), init(nn.Linear(self.HIDDEN, 1)))
        self._flat = None

    @classmethod
    def from_shapes(cls, obs_shape, n_actions: int) -> "DuelingDQN":
        return cls(env_spec(obs_shape, n_actions))

    def forward(self, x):
        h = self.flatten(self.features(x))
        adv = self.advantage(h)
        val = self.value(h)
        return val + adv - adv.mean(1, keepdim=True)

    def _feature_size(self):
        with torch.no_grad():
            return self.features(torch.zeros(1, *self.input_shape)).view(1, -1).size(1)

    def act(self, state, epsilon):
        """(int action, float32[A] Q) for one state; epsilon-greedy via ``random``."""
        with torch.no_grad():
            q = self.forward(state.unsqueeze(0))
            if random.random() > epsilon:
                action = q.max(1)[1].item()
            else:
                action = random.randrange(self.num_actions)
        return action, q.cpu().numpy()[0]

    # -- flat parameter buffer ------------------------------------------------------
    def flatten_parameters(self) -> torch.Tensor:
        """Re-seat all parameters as views of one contiguous fp32 buffer (idempotent)."""
        params = list(self.parameters())
        if self._flat is not None:
            sp = self._flat.untyped_storage().data_ptr()
            if all(p.data.untyped_storage().data_ptr() == sp for p in params):
                return self._flat
        total = sum(p.numel() for p in params)
        flat = torch.empty(total, dtype=torch.float32, device=params[0].device)
        off = 0
        for p in params:
            n = p.numel()
            flat[off:off + n].copy_(p.data.reshape(-1))
            p.data = flat[off:off + n].view_as(p.data)
            off += n
        self._flat = flat
        return flat

    def param_segments(self) -> list[tuple[str, int, int]]:
        """(name, offset, numel) of each parameter inside the flat buffer."""
        out, off = [], 0
        for name, p in self.named_parameters():
            out.append((name, off, p.numel()))
            off += p.numel()
        return out
