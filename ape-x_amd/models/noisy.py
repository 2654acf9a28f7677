"""Factorised-Gaussian NoisyNet linear layer (reference model.py:112-164).

``weight_mu/sigma`` and ``bias_mu/sigma`` are parameters; ``weight_epsilon`` and
``bias_epsilon`` are *buffers* (so they live in the state_dict, as in the
reference checkpoint format).  Train mode uses mu + sigma * eps, eval uses mu.
Init: mu ~ U(+-1/sqrt(in)), sigma = std_init/sqrt(fan) ; noise f(x)=sign(x)sqrt|x|,
eps_w = f(eps_out) outer f(eps_in), eps_b = fresh f(eps_out).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


class NoisyLinear(nn.Module):
    def __init__(self, in_features, out_features, device=None, std_init=0.4):
        super().__init__()
        self.device = device
        self.in_features = in_features
        self.out_features = out_features
        self.std_init = std_init
        self.weight_mu = nn.Parameter(torch.empty(out_features, in_features))
        self.weight_sigma = nn.Parameter(torch.empty(out_features, in_features))
        self.register_buffer("weight_epsilon", torch.empty(out_features, in_features))
        self.bias_mu = nn.Parameter(torch.empty(out_features))
        self.bias_sigma = nn.Parameter(torch.empty(out_features))
        self.register_buffer("bias_epsilon", torch.empty(out_features))
        self.reset_parameters()
        self.reset_noise()

    def forward(self, x):
        if self.training:
            w = torch.addcmul(self.weight_mu, self.weight_sigma, self.weight_epsilon.to(self.weight_mu.device))
            b = torch.addcmul(self.bias_mu, self.bias_sigma, self.bias_epsilon.to(self.bias_mu.device))
        else:
            w, b = self.weight_mu, self.bias_mu
        return F.linear(x, w, b)

    def reset_parameters(self):
        bound = 1.0 / math.sqrt(self.weight_mu.size(1))
        with torch.no_grad():
            self.weight_mu.uniform_(-bound, bound)
            self.weight_sigma.fill_(self.std_init / math.sqrt(self.weight_sigma.size(1)))
            self.bias_mu.uniform_(-bound, bound)
            self.bias_sigma.fill_(self.std_init / math.sqrt(self.bias_sigma.size(0)))

    @staticmethod
    def _scale_noise(size):
        x = torch.randn(size)
        return x.sign().mul(x.abs().sqrt())

    def reset_noise(self):
        eps_in = self._scale_noise(self.in_features)
        eps_out = self._scale_noise(self.out_features)
        with torch.no_grad():
            self.weight_epsilon.copy_(torch.outer(eps_out, eps_in))
            self.bias_epsilon.copy_(self._scale_noise(self.out_features))

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, std_init={self.std_init}"
