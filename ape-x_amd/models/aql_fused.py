"""HIP fast path of the AQL model: batched candidate proposal, candidate
Q evaluation and epsilon-greedy selection as three gfx950 kernels.

``FusedAQL(model)`` reads the weights of an :class:`~apex_amd.models.aql.AQL` in place (no
copies; NoisyLinear noise buffers included) and offers

* ``candidate_q(state, a_mu)`` -> Q [B, T] (no grad): the critic over the candidate set,
  fused (q_feature, action encoder, concat, NoisyLinear x2) -- used for the two no-grad
  evaluations of the AQL loss (online and target Q at s') and by batched actors;
* ``propose(state)`` -> a_mu: uniform + proposal samples drawn on device (Philox);
* ``act(state, eps)`` -> (candidate index, a_mu, env action) for a batch of envs: the
  batched version of ``AQL.act`` (reference model.py:198-205), one launch each.

Numerics are fp32 (the MLPs are tiny; the win is launch count and no host round trip:
the reference's ``AQL.act`` runs ~20 small torch ops plus a ``.cpu()`` per env step).
"""
from __future__ import annotations

import torch

from .. import ops
from .aql import AQL


class FusedAQL:
    def __init__(self, model: AQL, seed: int = 0):
        self.hip = ops.hip()
        self.model = model
        q, pr = model.q, model.proposal
        self.device = next(model.parameters()).device
        assert self.device.type == "cuda", "FusedAQL needs the model on the GPU"
        self.cont = bool(model.env_iscontinuous)
        self.na = int(model.num_actions)
        self.adim = self.na if self.cont else 1
        self.T = int(model.total_sample)
        self.obs = int(model.input_shape[0])
        self.seed = int(seed)
        f32 = dict(dtype=torch.float32, device=self.device)
        self.ws = torch.empty(self.hip.aql_workspace_floats(), **f32)
        self.counter = torch.zeros(1, dtype=torch.int64, device=self.device)
        if self.cont:
            space = model.env.action_space
            self.low = torch.as_tensor(space.low, **f32).reshape(-1).contiguous()
            self.high = torch.as_tensor(space.high, **f32).reshape(-1).contiguous()
            self.var = pr.action_var.to(**f32).contiguous()
        else:
            self.low = self.high = self.var = torch.zeros(1, **f32)
        a1, a2 = q.advantage1, q.advantage2
        self._tensors = {
            "qf_w1": q.q_feature[0].weight, "qf_b1": q.q_feature[0].bias,
            "qf_w2": q.q_feature[2].weight, "qf_b2": q.q_feature[2].bias,
            "ao_w1": q.action_out[0].weight, "ao_b1": q.action_out[0].bias,
            "a1_wmu": a1.weight_mu, "a1_wsig": a1.weight_sigma, "a1_weps": a1.weight_epsilon,
            "a1_bmu": a1.bias_mu, "a1_bsig": a1.bias_sigma, "a1_beps": a1.bias_epsilon,
            "a2_wmu": a2.weight_mu, "a2_wsig": a2.weight_sigma, "a2_weps": a2.weight_epsilon,
            "a2_bmu": a2.bias_mu, "a2_bsig": a2.bias_sigma, "a2_beps": a2.bias_epsilon,
            "f_w": q.features[0].weight, "f_b": q.features[0].bias,
            "df_w1": pr.dist_feature[0].weight, "df_b1": pr.dist_feature[0].bias,
            "df_w2": pr.dist_feature[2].weight, "df_b2": pr.dist_feature[2].bias,
        }
        if self.cont:
            self._tensors["ao_w2"] = q.action_out[2].weight
            self._tensors["ao_b2"] = q.action_out[2].bias
        self._cache = None

    def _net(self):
        noisy = int(self.model.q.training)
        ptrs = {k: int(t.data_ptr()) for k, t in self._tensors.items()}
        key = (noisy, tuple(ptrs.values()))
        if self._cache is None or self._cache[0] != key:
            for k, t in self._tensors.items():
                assert t.is_contiguous() and t.dtype == torch.float32 and t.device == self.device, k
            ints = dict(obs=self.obs, adim=self.adim, cont=int(self.cont), T=self.T, na=self.na,
                        uniform=int(self.model.uniform_sample), propose=int(self.model.propose_sample), noisy=noisy)
            self._cache = (key, self.hip.make_aql_net(ints, ptrs))
        return self._cache[1]

    @staticmethod
    def _s() -> int:
        return torch.cuda.current_stream().cuda_stream

    def _state(self, state) -> torch.Tensor:
        st = torch.as_tensor(state, dtype=torch.float32, device=self.device)
        return st.reshape(-1, self.obs).contiguous()

    def candidate_q(self, state, a_mu: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        st = self._state(state)
        B = st.shape[0]
        am = a_mu.to(device=self.device, dtype=torch.float32).contiguous()
        assert am.numel() == B * self.T * self.adim, "a_mu must be [B, T(, action_dim)]"
        q = out if out is not None else torch.empty(B, self.T, dtype=torch.float32, device=self.device)
        self.hip.aql_candidate_q(self._net(), self.ws.data_ptr(), st.data_ptr(), am.data_ptr(), B, q.data_ptr(),
                                 self._s())
        return q

    def propose(self, state, a_mu: torch.Tensor | None = None, bump: bool = True) -> torch.Tensor:
        st = self._state(state)
        B = st.shape[0]
        shape = (B, self.T, self.na) if self.cont else (B, self.T)
        am = a_mu if a_mu is not None else torch.empty(shape, dtype=torch.float32, device=self.device)
        self.hip.aql_propose(self._net(), st.data_ptr(), B, self.low.data_ptr(), self.high.data_ptr(),
                             self.var.data_ptr(), self.seed, self.counter.data_ptr(), am.data_ptr(), 0, self._s())
        if bump:
            self.counter.add_(1)
        return am

    def act(self, state, eps: torch.Tensor | float):
        """Batched epsilon-greedy over freshly proposed candidates.  Returns
        (candidate index int32 [B], a_mu, env action [B, action_dim] (cont) / [B] (disc))."""
        st = self._state(state)
        B = st.shape[0]
        am = self.propose(st, bump=False)
        q = self.candidate_q(st, am)
        eps_t = eps if isinstance(eps, torch.Tensor) else torch.full((B,), float(eps), device=self.device)
        idx = torch.empty(B, dtype=torch.int32, device=self.device)
        env_act = torch.empty(B, self.adim, dtype=torch.float32, device=self.device)
        self.hip.aql_select(q.data_ptr(), am.data_ptr(), B, self.T, self.adim, eps_t.contiguous().data_ptr(),
                            self.seed ^ 0xA9C1, self.counter.data_ptr(), idx.data_ptr(), env_act.data_ptr(),
                            self._s())
        self.counter.add_(1)
        return idx, am, (env_act if self.cont else env_act.reshape(B))
