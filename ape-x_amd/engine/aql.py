"""GPU AQL engine: distributed-actor Amortized Q-Learning with everything on one MI355X
(BASELINE config 4; reference AQL_dis.py:18-170, batchrecoder_AQL.py:13-138,
utils.py:44-61, model.py:112-390, memory.py:364-391).

What runs where (all device-side, no host sync inside an iteration):

* ``E`` vectorised GPU envs (``aql_env_step``: BipedalWalker-shaped / CartPole / Pendulum
  dynamics of :mod:`apex_amd.envs.classic`) act with a published copy of the online
  network: on-device candidate proposal (``aql_propose``: uniform + MVN / Categorical on
  Philox), the fused candidate critic (``aql_candidate_q``) and per-env epsilon-greedy
  selection (``aql_select``) with the reference worker ladder eps_i = 0.4^(1 + 7 i/(N-1))
  (batchrecoder_AQL.py:97-99).  Each step inserts the raw (s, a, r, s', d, a_mu)
  transitions into the HBM replay ring at max priority (no n-step, no actor priorities:
  batchrecoder_AQL.py:48-51; the 24x duplicate insert of the reference, Q8, is not
  reproduced).
* :class:`AQLReplay`: tables ``[C, obs]`` x2, action/reward/done ``[C]``, the candidate
  sets ``a_mu [C, T, adim]`` and the fanout-64 HBM priority tree shared with the DQN
  engine (``per_*`` kernels).
* One learner step (``AQLLearner.step``; AQL_dis.py:63-108) = stratified PER sample ->
  ``aql_learn_fwd`` (online Q(s,.), Q(s',.), target Q(s',.) over the stored candidates,
  fp32 MFMA) -> ``aql_learn_bwd`` (Double-Q Huber TD, proposal log-prob/entropy loss,
  backward vectors) -> priority write (0.9 max + 0.1 |td| + 1e-6 mix, fused) ->
  ``aql_grad`` (both losses' weight gradients + per-group norms) -> two Adam steps with
  separate clip_grad_norm_(40) (critic, proposal) -> ``aql_post`` (reset_noise() of the
  online and target NoisyNets + proposal hard copy online -> target, AQL_dis.py:92,104-105).
  K learner steps are captured in one hipGraph.

Iteration = one actor step of all E envs + ``E // batch`` learner steps: the reference's
replay ratio (``total_ep_len // batch_size`` SGD steps per recorded batch, AQL_dis.py:118).
Weights are published to the actors every iteration (set_worker_weights, AQL_dis.py:115)
and the target network is synced after the learner steps of every iteration whose index is
a multiple of ``target_update_interval`` -- iteration 0 included (AQL_dis.py:127-129);
``target_update_steps > 0`` switches to a learner-step cadence instead (round-2 default).

Reference behaviours kept: q.features (the state embedding feeding the proposal) receives
gradient only from the proposal loss, which optimizer_q zeroes before its own backward, so
it never changes (its Adam step sees a None/zero gradient); the discrete proposal loss
broadcasts log_prob([B,1]) against batch [B] (see aql_engine_kernels.hip).
"""
from __future__ import annotations

import collections
import math
from dataclasses import dataclass

import numpy as np
import torch

from .. import envs, ops
from ..algo.schedules import actor_epsilon
from ..models.aql import AQL
from ..models.aql_fused import FusedAQL
from .hbm_replay import tree_level_sizes

ENV_KINDS = {"BipedalWalker-v3": 0, "CartPole-v0": 1, "CartPole-v1": 1, "Pendulum-v0": 2, "Pendulum-v1": 2}


def flatten_module_params(module: torch.nn.Module, align: int = 4) -> torch.Tensor:
    """Re-seat every parameter of ``module`` as a view of one contiguous fp32 buffer
    (named_parameters order), each starting at a multiple of ``align`` floats (16-byte rows
    for the learner's vector loads; the zero gaps get zero gradients and stay zero).
    Offsets are kept in ``module._flat_offsets``; returns the buffer."""
    params = list(module.named_parameters())
    offs, off = {}, 0
    for name, p in params:
        off = -(-off // align) * align
        offs[name] = off
        off += p.numel()
    flat = torch.zeros(-(-off // align) * align, dtype=torch.float32, device=params[0][1].device)
    for name, p in params:
        o, n = offs[name], p.numel()
        flat[o:o + n].copy_(p.data.reshape(-1))
        p.data = flat[o:o + n].view_as(p.data)
    module._flat_offsets = offs
    return flat


def flatten_noise(model: AQL) -> torch.Tensor:
    """Re-seat the four NoisyLinear epsilon buffers of ``model.q`` as views of one buffer:
    [advantage1.weight_epsilon, advantage1.bias_epsilon, advantage2.weight_epsilon,
    advantage2.bias_epsilon]."""
    bufs = [model.q.advantage1.weight_epsilon, model.q.advantage1.bias_epsilon,
            model.q.advantage2.weight_epsilon, model.q.advantage2.bias_epsilon]
    flat = torch.empty(sum(b.numel() for b in bufs), dtype=torch.float32, device=bufs[0].device)
    off = 0
    for b in bufs:
        n = b.numel()
        flat[off:off + n].copy_(b.reshape(-1))
        b.data = flat[off:off + n].view_as(b)
        off += n
    return flat


class AQLReplay:
    """HBM prioritized replay with candidate sets (reference CustomPrioritizedReplayBuffer_AQL,
    memory.py:364-391): insert at max priority, proportional stratified sampling with IS
    weights, priorities**alpha in the fanout-64 device tree."""

    def __init__(self, capacity: int, obs: int, T: int, adim: int, alpha: float = 0.6,
                 device: str | torch.device = "cuda", seed: int = 0):
        self.hip = ops.hip()
        self.device = torch.device(device)
        self.capacity, self.obs, self.T, self.adim = int(capacity), int(obs), int(T), int(adim)
        self.alpha, self.seed = float(alpha), int(seed)
        C, dev = self.capacity, self.device
        f32 = dict(dtype=torch.float32, device=dev)
        self.st = torch.zeros(C, obs, **f32)
        self.st2 = torch.zeros(C, obs, **f32)
        self.action = torch.zeros(C, dtype=torch.int32, device=dev)
        self.reward = torch.zeros(C, **f32)
        self.done = torch.zeros(C, **f32)
        self.a_mu = torch.zeros(C, T, adim, **f32)
        sizes = tree_level_sizes(C)
        self.level_sizes = sizes
        self.leaf_sum = torch.zeros(C, **f32)
        self.leaf_min = torch.full((C,), math.inf, **f32)
        self.node_sum = [torch.zeros(n, dtype=torch.float64, device=dev) for n in sizes[1:]]
        self.node_min = [torch.full((n,), math.inf, **f32) for n in sizes[1:]]
        self.max_prio = torch.ones(1, **f32)
        self.filled = torch.zeros(1, dtype=torch.int64, device=dev)
        self.sorted_scratch = torch.zeros(1024, dtype=torch.int32, device=dev)
        # batched tree write scratch (per_write_batch): dedup claims (-1 between writes),
        # dirty-slot list, last-block ticket
        self.owner = torch.full((C,), -1, dtype=torch.int32, device=dev)
        self.wlist = torch.zeros(2048, dtype=torch.int32, device=dev)
        self.ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        self.tree = self.hip.make_tree(self.leaf_sum.data_ptr(), self.leaf_min.data_ptr(),
                                       [t.data_ptr() for t in self.node_sum], [t.data_ptr() for t in self.node_min],
                                       sizes)

    def nbytes(self) -> int:
        ts = [self.st, self.st2, self.action, self.reward, self.done, self.a_mu, self.leaf_sum, self.leaf_min,
              *self.node_sum, *self.node_min]
        return sum(t.numel() * t.element_size() for t in ts)

    def table_ptrs(self) -> dict:
        return {"st": self.st.data_ptr(), "st2": self.st2.data_ptr(), "rew": self.reward.data_ptr(),
                "done": self.done.data_ptr(), "amu": self.a_mu.data_ptr(), "act": self.action.data_ptr()}

    def __len__(self) -> int:
        return int(min(self.filled.item(), self.capacity))

    def total_priority(self) -> float:
        return float(self.node_sum[-1][0].item())


@dataclass
class AQLEngineConfig:
    env_id: str = "BipedalWalker-v3"
    n_envs: int = 256
    capacity: int = 1_000_000
    batch_size: int = 32
    gamma: float = 0.99
    n_steps: int = 1
    lr: float = 1e-3
    ent_lam: float = 0.8
    propose_sample: int = 1
    uniform_sample: int = 50
    action_var: float = 0.25
    alpha: float = 0.6
    beta_start: float = 0.4
    max_step: int = 1_000_000      # beta annealing horizon, in iterations (AQL_dis.py:59)
    n_workers: int = 10            # the reference's beta-annealing factor (AQL_dis.py:59)
    max_norm: float = 40.0
    learner_steps: int | None = None   # per iteration; None = n_envs // batch_size
    target_update_interval: int = 20   # iterations between target syncs, iteration 0 included (AQL_dis.py:127)
    target_update_steps: int = 0       # > 0: sync every this many learner steps instead (not the reference's)
    track_losses: bool = False         # accumulate loss_q / loss_proposal per step on device (train CLI logging)
    eps_base: float = 0.4
    eps_alpha: float = 7.0
    total_actors: int | None = None    # epsilon ladder width (multi-GPU: all actors)
    actor_offset: int = 0
    threshold: int | None = None       # transitions before learning (default batch_size + 1)
    exact_mass: bool = False           # False = reference sampling mass (Q5)
    use_graphs: bool = True
    # The learner step's launch sequence.  True (default): four launches per SGD step --
    #   aql_learn_fwd   (draws its own PER rows, or uses the rows the previous step drew)
    #   aql_learn_bwd   (+ one workgroup: priority mix, loss mean, deduplicated leaves, tree level 1)
    #   aql_grad        (+ one workgroup: tree levels 2..)
    #   aql_update      (both clipped Adam steps, noise reset of both critics, proposal copy,
    #                    step bump, the NEXT step's PER draw; the iteration's last step also
    #                    writes the acting copies)
    # MI355X, batch 32: 19.0k SGD steps/s (profiles/archive_r4.md (r4_aql_engine.md)).  False: the reference
    # sequence of separate launches (per_sample, forward, backward, per_write_batch, gradients,
    # adam_step2, noise reset) -- the bit-identity baseline of tests/test_gpu_aql_engine.py.
    # (Round 4 alternatives measured slower and removed: a forked tree stream, the whole step
    # tail in one grid-barrier launch, the tree write in the noise-reset launch.)
    fused: bool = True
    # acting on its own HIP stream beside the learner steps (staged transitions); MI355X, B 32:
    # 12978-13005 vs 13161 SGD steps/s serial -- the learner's chain of small kernels slows by
    # about what the hidden acting step saves, so serial stays the default
    overlap: bool = False
    # learner forward: candidate-tile groups per (sample, net) workgroup (0 = about one workgroup
    # per CU: the ~110 KB weight staging, the PER draw and the state MLP serve a group of tiles)
    fwd_tile_groups: int = 0
    # serial acting tail in one launch (aql_act_tail: eps-greedy select + env step + ring tree
    # write + counter bumps + the learner's PER beta) instead of select, env step, ring write
    # and a host beta fill; False = the separate launches (the bit-identity baseline)
    fused_acting: bool = True
    seed: int = 0


def target_sync_due(cfg: AQLEngineConfig, iteration: int, steps_before: int, steps_after: int) -> bool:
    """Whether the full online -> target copy follows the learner steps of ``iteration``.
    Reference cadence: ``frame_idx % target_update_interval == 0`` after that iteration's
    SGD loop (AQL_dis.py:127-129), so iteration 0 syncs.  ``target_update_steps > 0``:
    whenever the learner-step count crosses a multiple of it."""
    tu = int(cfg.target_update_steps)
    if tu > 0:
        return steps_before // tu != steps_after // tu
    ti = int(cfg.target_update_interval)
    return ti > 0 and iteration % ti == 0


class AQLLearner:
    """Device-resident AQL learner over an :class:`AQLReplay` (see module docstring)."""

    def __init__(self, model: AQL, target: AQL, replay: AQLReplay, cfg: AQLEngineConfig):
        self.hip = h = ops.hip()
        self.cfg, self.model, self.target, self.replay = cfg, model, target, replay
        dev = replay.device
        self.device = dev
        self.flat = flatten_module_params(model)
        self.tflat = flatten_module_params(target)
        self.eps = flatten_noise(model)
        self.teps = flatten_noise(target)
        names = [n for n, _ in model.named_parameters()]
        n_q = sum(1 for n in names if n.startswith("q."))
        assert all(n.startswith("q.") for n in names[:n_q]) and n_q < len(names), \
            "critic parameters must precede the proposal's in the flat layout"
        self.P = self.flat.numel()
        self.P_q = model._flat_offsets[names[n_q]]  # first proposal parameter (aligned)
        self.P_p = self.P - self.P_q
        B, T = cfg.batch_size, model.total_sample
        self.B, self.T = B, T
        f32 = dict(dtype=torch.float32, device=dev)
        self.idx = torch.zeros(B, dtype=torch.int32, device=dev)
        self.w = torch.zeros(B, **f32)
        self.q_s = torch.zeros(B, T, **f32)
        self.q_s2 = torch.zeros(B, T, **f32)
        self.qt_s2 = torch.zeros(B, T, **f32)
        lay = h.aql_vec_layout()
        self.lay = lay
        self.vec = torch.zeros(B, lay["STRIDE"], **f32)
        self.delta = torch.zeros(B, **f32)
        self.lw = torch.zeros(B, **f32)
        self.lossp = torch.zeros(B, **f32)
        self.prio = torch.zeros(B, **f32)
        self.loss_q = torch.zeros(1, **f32)
        self.loss_p = torch.zeros(1, **f32)
        self.loss_acc = torch.zeros(3, dtype=torch.float64, device=dev)  # sum loss_q, sum loss_p, steps
        self._acc_one = torch.ones(1, dtype=torch.float64, device=dev)
        self.grad = torch.zeros(self.P, **f32)
        self.m = torch.zeros(self.P, **f32)
        self.v = torch.zeros(self.P, **f32)
        self.nblk = h.aql_grad_blocks(self.P)
        self.part = torch.zeros(2 * self.nblk, dtype=torch.float64, device=dev)
        self.norms_q = torch.zeros(4, **f32)
        self.norms_p = torch.zeros(4, **f32)
        self.step_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        self.ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        self.beta = torch.full((1,), cfg.beta_start, **f32)
        self.var = model.proposal.action_var.to(**f32).contiguous()
        self.hp = h.AdamParams(cfg.lr, max_norm=cfg.max_norm)
        self.fused_on = FusedAQL(model)
        self.fused_tg = FusedAQL(target)
        nws = h.aql_workspace_floats()  # effective NoisyLinear weights: W1 [64][128] | b1 | w2 | b2
        self.eff_on = torch.zeros(nws, **f32)
        self.eff_tg = torch.zeros(nws, **f32)
        p = dict(replay.table_ptrs(), eff_on=self.eff_on.data_ptr(), eff_tg=self.eff_tg.data_ptr(), idx=self.idx.data_ptr(), w=self.w.data_ptr(), var=self.var.data_ptr(),
                 q_s=self.q_s.data_ptr(), q_s2=self.q_s2.data_ptr(), qt_s2=self.qt_s2.data_ptr(),
                 vec=self.vec.data_ptr(), delta=self.delta.data_ptr(), lw=self.lw.data_ptr(),
                 lossp=self.lossp.data_ptr())
        self.L = h.make_aql_learn(self.fused_on._net(), self.fused_tg._net(), p, B,
                                  float(cfg.gamma ** cfg.n_steps), float(cfg.ent_lam))
        if cfg.fwd_tile_groups:
            self.L = h.aql_learn_set_groups(self.L, int(cfg.fwd_tile_groups), 0)
        self.G = h.make_aql_grad(self._grad_jobs(), self.P, self.vec.data_ptr(), B, self.grad.data_ptr(),
                                 self.part.data_ptr(), self.lossp.data_ptr(), self.loss_p.data_ptr())
        layers = []
        for m, eff in ((model, self.eff_on), (target, self.eff_tg)):
            n1 = 64 * 128
            views = ((eff[:n1], eff[n1:n1 + 64]), (eff[n1 + 64:n1 + 128], eff[n1 + 128:n1 + 129]))
            for lin, (weff, beff) in zip((m.q.advantage1, m.q.advantage2), views):
                assert weff.numel() == lin.weight_mu.numel() and beff.numel() == lin.bias_mu.numel()
                layers.append((lin.weight_epsilon.data_ptr(), lin.bias_epsilon.data_ptr(), lin.weight_mu.data_ptr(),
                               lin.weight_sigma.data_ptr(), lin.bias_mu.data_ptr(), lin.bias_sigma.data_ptr(),
                               weff.data_ptr(), beff.data_ptr(), lin.out_features, lin.in_features))
        self.post = h.make_aql_post(layers, self.flat[self.P_q:].data_ptr(), self.tflat[self.P_q:].data_ptr(),
                                    self.P_p, self.step_ctr.data_ptr(), self.ticket.data_ptr(),
                                    (cfg.seed * 0x9E3779B1 + 0x5EED) & 0xFFFFFFFFFFFF)
        r = replay
        self.fused = bool(cfg.fused) and B <= 64  # (the tree workgroups stage <= 64 dirty paths)
        self.Ls = self.L_tree = self.G_levels = self.U = self.U_draw = self.U_pub = None
        self.U_gate = self.U_gate_draw = self._gate_ptr = None
        if self.fused:
            # the forward's own stratified draw (same seed, counter and mass as per_sample)
            self.Ls = h.aql_learn_set_sample(self.L, r.tree, r.filled.data_ptr(), self.beta.data_ptr(),
                                             self.step_ctr.data_ptr(), r.seed ^ 0x51A7, 0 if cfg.exact_mass else 1)
            # the backward's extra workgroup recomputes the B TD terms from the forward's Q rows and
            # writes the priorities (0.9 max + 0.1 |td| + 1e-6), the loss mean, the deduplicated
            # leaves and tree level 1; the gradient launch's extra workgroup walks levels 2..
            self.L_tree = h.aql_learn_set_tree(self.L, r.tree, self.prio.data_ptr(), self.loss_q.data_ptr(),
                                               r.owner.data_ptr(), r.wlist.data_ptr(), r.max_prio.data_ptr(), r.alpha,
                                               levels=1)
            # the gradient launch snapshots the step counter for the update launch, which then
            # bumps it from one workgroup instead of a last-workgroup ticket
            self.step_snap = torch.zeros(1, dtype=torch.int64, device=dev)
            self.G = h.aql_grad_set_step_snap(self.G, self.step_snap.data_ptr(), self.step_ctr.data_ptr())
            self.G_levels = h.aql_grad_set_levels(self.G, r.tree, r.wlist.data_ptr(), B, lo=2)
            kw = dict(p=self.flat.data_ptr(), m=self.m.data_ptr(), v=self.v.data_ptr(), n=self.P, P_q=self.P_q,
                      norms_q=self.norms_q.data_ptr(), norms_p=self.norms_p.data_ptr(), update=1)
            nb = h.aql_step_nbytes()
            self.step_desc = torch.zeros(2, nb, dtype=torch.uint8, device=dev)
            self.pub_desc = torch.zeros(nb, dtype=torch.uint8, device=dev)
            self._step_kw = kw
            self.U = h.make_aql_step(self.L, self.G, self.post, r.tree, self.hp, kw, self.step_desc[0].data_ptr())
            # + the NEXT step's draw (the tree is final once the backward launch's write is done)
            self.U_draw = h.make_aql_step(self.L, self.G, self.post, r.tree, self.hp,
                                          dict(kw, draw=1, filled=r.filled.data_ptr(), beta=self.beta.data_ptr(),
                                               seed=r.seed ^ 0x51A7, exclude_last=0 if cfg.exact_mass else 1),
                                          self.step_desc[1].data_ptr())
        self.refresh()

    def set_publish(self, actor_flat: torch.Tensor, actor_eps: torch.Tensor) -> None:
        """The iteration's last step can write the acting copies (weights + online noise) from
        its update launch (``step(publish=True)``) instead of two copy launches after it."""
        if self.U is None:
            return
        e0 = self.eps.data_ptr()
        sub = lambda buf: actor_eps.data_ptr() + (buf.data_ptr() - e0)  # noqa: E731
        a1, a2 = self.model.q.advantage1, self.model.q.advantage2
        assert actor_flat.numel() == self.P and actor_eps.numel() == self.eps.numel()
        self._pub_keep = (actor_flat, actor_eps)
        self.U_pub = self.hip.make_aql_step(
            self.L, self.G, self.post, self.replay.tree, self.hp,
            dict(self._step_kw, update=1, pub_p=actor_flat.data_ptr(), pub_weps0=sub(a1.weight_epsilon),
                 pub_beps0=sub(a1.bias_epsilon), pub_weps1=sub(a2.weight_epsilon), pub_beps1=sub(a2.bias_epsilon)),
            self.pub_desc.data_ptr())

    def _make_gated(self, gate: torch.Tensor) -> None:
        """Update-launch descriptors that honour the step gate ``gate``."""
        r = self.replay
        kw = dict(self._step_kw, gate=gate.data_ptr())
        self._gate_ptr, self._gate_keep = gate.data_ptr(), gate
        self.gate_desc = torch.zeros_like(self.step_desc)
        self.U_gate = self.hip.make_aql_step(self.L, self.G, self.post, r.tree, self.hp, kw,
                                             self.gate_desc[0].data_ptr())
        self.U_gate_draw = self.hip.make_aql_step(
            self.L, self.G, self.post, r.tree, self.hp,
            dict(kw, draw=1, filled=r.filled.data_ptr(), beta=self.beta.data_ptr(), seed=r.seed ^ 0x51A7,
                 exclude_last=0 if self.cfg.exact_mass else 1), self.gate_desc[1].data_ptr())

    @property
    def predraw(self) -> bool:
        """Whether a step can draw the next step's rows (the fused sequence's update launch)."""
        return self.U_draw is not None

    def refresh(self) -> None:
        """Recompute the effective NoisyLinear weights (mu + sigma * eps) of both networks
        from their current parameters / noise: after init, a target sync or any direct
        parameter edit (load_state_dict)."""
        self.hip.aql_post(self.post, 0, self._s())

    def _grad_jobs(self):
        lay, m = self.lay, self.model
        cont = m.env_iscontinuous
        a1, a2 = m.q.advantage1, m.q.advantage2
        spec = {
            "q.q_feature.0.weight": ("GQFH", "S", None), "q.q_feature.0.bias": ("GQFH", None, None),
            "q.q_feature.2.weight": ("GX+", "QFH", None), "q.q_feature.2.bias": ("GX+", None, None),
            "q.action_out.0.weight": ("GAOH" if cont else "GX", "A", None),
            "q.action_out.0.bias": ("GAOH" if cont else "GX", None, None),
            "q.action_out.2.weight": ("GX", "AOH", None), "q.action_out.2.bias": ("GX", None, None),
            "q.advantage1.weight_mu": ("GH", "X", None), "q.advantage1.weight_sigma": ("GH", "X", a1.weight_epsilon),
            "q.advantage1.bias_mu": ("GH", None, None), "q.advantage1.bias_sigma": ("GH", None, a1.bias_epsilon),
            "q.advantage2.weight_mu": ("GQ", "H", None), "q.advantage2.weight_sigma": ("GQ", "H", a2.weight_epsilon),
            "q.advantage2.bias_mu": ("GQ", None, None), "q.advantage2.bias_sigma": ("GQ", None, a2.bias_epsilon),
            "proposal.dist_feature.0.weight": ("GHID", "EMB", None), "proposal.dist_feature.0.bias": ("GHID", None, None),
            "proposal.dist_feature.2.weight": ("GMU", "HID", None), "proposal.dist_feature.2.bias": ("GMU", None, None),
        }
        jobs, off = [], 0
        for name, p in m.named_parameters():
            o = m._flat_offsets[name]
            if o > off:  # alignment gap: zero gradient
                jobs.append((off, o - off, 1, 0, -1, 0, 0, 1))
                off = o
            rows = p.shape[0]
            cols = p.numel() // rows
            group = 1 if name.startswith("proposal.") else 0
            if name.startswith("q.features."):
                jobs.append((off, rows, cols, 0, -1, 0, group, 1))
            else:
                g, x, eps = spec[name]
                goff = lay["GX"] + 64 if g == "GX+" else lay[g]
                xoff = -1 if x is None else lay[x]
                if xoff < 0:
                    rows, cols = p.numel(), 1
                jobs.append((off, rows, cols, goff, xoff, 0 if eps is None else eps.data_ptr(), group, 0))
            off += p.numel()
        if off < self.P:
            jobs.append((off, self.P - off, 1, 0, -1, 0, 1, 1))
        return jobs

    @staticmethod
    def _s() -> int:
        return torch.cuda.current_stream().cuda_stream

    def step(self, drawn: bool = False, draw_next: bool = False, publish: bool = False,
             gate: torch.Tensor | None = None, j: int = 0) -> bool:
        """One SGD step.  ``drawn``: this step's rows were drawn by the previous step's update
        launch (``draw_next`` there) -- the forward skips its tree descent (:meth:`AQLEngine.
        learn_steps` pairs them within an iteration).  ``publish``: the update launch also writes
        the acting copies (returns whether it did).  ``gate`` (int32 [1], device): the step is
        step ``j`` of its iteration and runs only if ``j < gate`` -- every launch of a gated-off
        step returns at once (the central learner's rows-applied replay ratio)."""
        h, r, s = self.hip, self.replay, self._s()
        if drawn or draw_next:
            assert self.predraw, "pre-drawn rows need the fused sequence"
        if self.fused:
            g = 0 if gate is None else gate.data_ptr()
            if g and (self.U_gate is None or self._gate_ptr != g):
                self._make_gated(gate)
            U, U_draw = (self.U_gate, self.U_gate_draw) if g else (self.U, self.U_draw)
            h.aql_learn_fwd(self.L if drawn else self.Ls, s, g, j)
            h.aql_learn_bwd(self.L_tree, s, g, j)
            h.aql_grad(self.G_levels, s, g, j)
            pub = publish and not draw_next and self.U_pub is not None and not g
            h.aql_update(U_draw if draw_next else (self.U_pub if pub else U), s, j)
            self._track_losses()
            return pub
        if gate is not None:
            raise ValueError("the step gate needs the fused launch sequence")
        # the reference sequence
        excl = 0 if self.cfg.exact_mass else 1
        h.per_sample(r.tree, self.B, r.filled.data_ptr(), 0, self.beta.data_ptr(), 0.0, r.seed ^ 0x51A7,
                     self.step_ctr.data_ptr(), self.idx.data_ptr(), self.w.data_ptr(), excl, s)
        h.aql_learn_fwd(self.L, s)
        h.aql_learn_bwd(self.L, s)
        # priorities 0.9 max|td| + 0.1 |td| + 1e-6 (utils.py:55) and the loss mean, written with the
        # batched tree kernels (leaves + one wide launch per big level; duplicates last-write-wins)
        h.per_write_batch(r.tree, 0, 0, 0, 0, self.idx.data_ptr(), 0, self.B, self.delta.data_ptr(),
                          self.lw.data_ptr(), self.prio.data_ptr(), self.loss_q.data_ptr(), 0, r.owner.data_ptr(),
                          r.wlist.data_ptr(), r.max_prio.data_ptr(), r.alpha, r.ticket.data_ptr(), s)
        h.aql_grad(self.G, s)
        Pq, o = self.P_q, 4 * self.P_q
        # the two optimizers (critic, proposal; own clip norms) in one launch
        h.adam_step2((self.flat.data_ptr(), self.grad.data_ptr(), self.m.data_ptr(), self.v.data_ptr(), Pq,
                      self.part.data_ptr(), self.nblk, self.norms_q.data_ptr()),
                     (self.flat.data_ptr() + o, self.grad.data_ptr() + o, self.m.data_ptr() + o,
                      self.v.data_ptr() + o, self.P_p, self.part.data_ptr() + 8 * self.nblk, self.nblk,
                      self.norms_p.data_ptr()),
                     self.hp, self.step_ctr.data_ptr(), s)
        h.aql_post(self.post, 1, s)
        self._track_losses()
        return False

    def _track_losses(self) -> None:
        if self.cfg.track_losses:  # device-side running sums; read (one sync) only when logging
            self.loss_acc[0:1].add_(self.loss_q)
            self.loss_acc[1:2].add_(self.loss_p)
            self.loss_acc[2:3].add_(self._acc_one)

    def take_loss_means(self) -> tuple[float, float, int]:
        """(mean loss_q, mean loss_proposal, steps) since the previous call; resets the sums."""
        q, p, n = (float(x) for x in self.loss_acc.tolist())
        self.loss_acc.zero_()
        n = int(round(n))
        return (q / n, p / n, n) if n else (float("nan"), float("nan"), 0)

    def sync_target(self) -> None:
        """update_target (AQL_dis.py:60-61): full state_dict copy, noise buffers included."""
        s = self._s()
        self.hip.copy_f32(self.tflat.data_ptr(), self.flat.data_ptr(), self.P, s)
        self.hip.copy_f32(self.teps.data_ptr(), self.eps.data_ptr(), self.eps.numel(), s)
        self.refresh()

    def stats(self) -> dict:
        return {"loss_q": float(self.loss_q.item()), "loss_proposal": float(self.loss_p.item()),
                "grad_norm_q": float(self.norms_q[0].item()), "grad_norm_proposal": float(self.norms_p[0].item()),
                "steps": int(self.step_ctr.item())}


class AQLEngine:
    """Actors + replay + learner of AQL_dis on one GPU (see module docstring)."""

    def __init__(self, cfg: AQLEngineConfig, device: str | torch.device = "cuda"):
        self.cfg = cfg
        self.device = dev = torch.device(device)
        self.hip = h = ops.hip()
        if cfg.env_id not in ENV_KINDS:
            raise ValueError(f"GPU AQL env must be one of {sorted(ENV_KINDS)}")
        self.kind = ENV_KINDS[cfg.env_id]
        self.host_env = envs.make(cfg.env_id)
        torch.manual_seed(cfg.seed)
        kw = dict(propose_sample=cfg.propose_sample, uniform_sample=cfg.uniform_sample, action_var=cfg.action_var,
                  device=dev)
        self.model = AQL(env=self.host_env, **kw).to(dev)
        self.target = AQL(env=self.host_env, **kw).to(dev)
        self.target.load_state_dict(self.model.state_dict())
        self.actor_model = AQL(env=self.host_env, **kw).to(dev)
        for m in (self.model, self.target, self.actor_model):
            m.q.train()
        self.cont = bool(self.model.env_iscontinuous)
        self.T = int(self.model.total_sample)
        self.obs = int(self.host_env.observation_space.shape[0])
        self.adim = int(self.model.num_actions) if self.cont else 1
        self.replay = AQLReplay(cfg.capacity, self.obs, self.T, self.adim, cfg.alpha, dev, seed=cfg.seed + 17)
        self.learner = AQLLearner(self.model, self.target, self.replay, cfg)
        self.actor_flat = flatten_module_params(self.actor_model)
        self.actor_eps = flatten_noise(self.actor_model)
        self.publish()
        E = cfg.n_envs
        self.E = E
        self.K = cfg.learner_steps if cfg.learner_steps is not None else max(1, E // cfg.batch_size)
        f32 = dict(dtype=torch.float32, device=dev)
        self.obs_buf = torch.zeros(E, self.obs, **f32)
        self.phys = torch.zeros(E, 4, **f32)
        self.ep_len = torch.zeros(E, dtype=torch.int32, device=dev)
        self.ep_ret = torch.zeros(E, **f32)
        self.ep_count = torch.zeros(1, dtype=torch.int32, device=dev)
        self.log_cap = 4096
        self.ep_log = torch.zeros(self.log_cap, 2, **f32)
        self.amu = torch.zeros(E, self.T, self.adim, **f32)
        self.qbuf = torch.zeros(E, self.T, **f32)
        self.act_idx = torch.zeros(E, dtype=torch.int32, device=dev)
        self.env_act = torch.zeros(E, self.adim, **f32)
        self.slots = torch.zeros(E, dtype=torch.int32, device=dev)
        self.actor_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        total = cfg.total_actors or E
        eps = actor_epsilon(np.arange(cfg.actor_offset, cfg.actor_offset + E), total, cfg.eps_base, cfg.eps_alpha)
        self.eps = torch.as_tensor(np.atleast_1d(eps), **f32)
        self.ws = torch.zeros(h.aql_workspace_floats(), **f32)
        if self.cont:
            sp = self.host_env.action_space
            self.low = torch.as_tensor(np.asarray(sp.low, dtype=np.float32).reshape(-1), **f32)
            self.high = torch.as_tensor(np.asarray(sp.high, dtype=np.float32).reshape(-1), **f32)
        else:
            self.low = self.high = torch.zeros(1, **f32)
        self.var = self.model.proposal.action_var.to(**f32).contiguous()
        if self.kind == 0:
            self.dynA = torch.as_tensor(self.host_env.unwrapped._A, **f32).contiguous()
            self.dynB = torch.as_tensor(self.host_env.unwrapped._B, **f32).contiguous()
            self.dynw = torch.as_tensor(self.host_env.unwrapped._w, **f32).contiguous()
        else:
            self.dynA = self.dynB = self.dynw = torch.zeros(1, **f32)
        self.seed = (cfg.seed * 0x2545F491 + 0xAC7) & 0xFFFFFFFFFFFF
        self.env = h.make_aql_env(dict(
            kind=self.kind, E=E, obs=self.obs, adim=self.adim, T=self.T,
            max_steps=int(getattr(self.host_env, "_max_episode_steps", None) or 1_000_000),
            obs_buf=self.obs_buf.data_ptr(), phys=self.phys.data_ptr(), ep_len=self.ep_len.data_ptr(),
            ep_ret=self.ep_ret.data_ptr(), dynA=self.dynA.data_ptr(), dynB=self.dynB.data_ptr(),
            dynw=self.dynw.data_ptr(), seed=self.seed, counter=self.actor_ctr.data_ptr(),
            ep_count=self.ep_count.data_ptr(), ep_log=self.ep_log.data_ptr(), log_cap=self.log_cap))
        self.ins = h.make_aql_insert(dict(self.replay.table_ptrs(), C=self.replay.capacity,
                                          filled=self.replay.filled.data_ptr(), slots=self.slots.data_ptr()))
        # overlap: the acting step writes its transitions into staging half h (rows 0..E-1);
        # the learner's graph applies the other half (the previous acting step's) to the ring
        # before its first sample, so acting never touches a table or tree the learner reads
        self.overlap = bool(cfg.overlap)
        # serial mode: the iteration's last SGD step writes the acting copies from its update
        # launch (no publish copies after it); overlap mode publishes after the acting step
        if not self.overlap:
            self.learner.set_publish(self.actor_flat, self.actor_eps)
        self._pub_in_graph = False
        self._half = 0
        if self.overlap:
            self._zero64 = torch.zeros(1, dtype=torch.int64, device=dev)
            self._stage_slots = torch.zeros(E, dtype=torch.int32, device=dev)
            self._stage = []
            self._stage_ins = []
            for _ in (0, 1):
                t = {"st": torch.zeros(E, self.obs, **f32), "st2": torch.zeros(E, self.obs, **f32),
                     "rew": torch.zeros(E, **f32), "done": torch.zeros(E, **f32),
                     "amu": torch.zeros(E, self.T, self.adim, **f32),
                     "act": torch.zeros(E, dtype=torch.int32, device=dev)}
                self._stage.append(t)
                self._stage_ins.append(h.make_aql_insert(dict({k: v.data_ptr() for k, v in t.items()}, C=E,
                                                              filled=self._zero64.data_ptr(),
                                                              slots=self._stage_slots.data_ptr())))
            self._astream = torch.cuda.Stream(device=dev)
            self._ev_actor = [torch.cuda.Event(), torch.cuda.Event()]
            self._ev_learn = torch.cuda.Event()
        # the serial engine's fused acting tail (aql_act_tail); it also writes the learner's PER
        # beta for the iteration from a device iteration counter (AQL_dis.py:59)
        self._tail = None
        if cfg.fused_acting and not self.overlap and E <= 1024:
            r = self.replay
            self._ticket = torch.zeros(1, dtype=torch.int32, device=dev)
            self._iter_dev = torch.zeros(1, dtype=torch.int64, device=dev)
            self._tail = h.make_aql_tail(self.env, self.ins, r.tree, dict(
                q=self.qbuf.data_ptr(), amu=self.amu.data_ptr(), eps=self.eps.data_ptr(), sel_seed=self.seed ^ 0xA9C1,
                act_idx=self.act_idx.data_ptr(), env_act=self.env_act.data_ptr(), alpha=float(r.alpha),
                max_prio=r.max_prio.data_ptr(), filled=r.filled.data_ptr(), counter=self.actor_ctr.data_ptr(),
                ticket=self._ticket.data_ptr(), beta_out=self.learner.beta.data_ptr(), iter=self._iter_dev.data_ptr(),
                beta0=float(cfg.beta_start), beta_omb=1.0 - cfg.beta_start, beta_max_step=float(cfg.max_step),
                beta_workers=float(cfg.n_workers)))
        self.actor_net = FusedAQL(self.actor_model)._net()
        # acting on the learner's MFMA candidate forward (online net, s only, row = env index)
        # (64 acting workgroups beside the learner in overlap mode: most CUs stay the learner's)
        self.actL = h.make_aql_act(self.actor_net, self.obs_buf.data_ptr(), self.amu.data_ptr(), self.ws.data_ptr(),
                                   self.qbuf.data_ptr(), E, 64 if cfg.overlap else 0)
        h.aql_env_reset(self.env, self._s())
        self._iterations = 0
        self.learner_steps = 0
        self._g_actor = self._g_learn = self._g_iter = None
        self._ep_read = 0
        self.target_syncs = collections.deque(maxlen=4096)  # iterations after which the target was synced

    @staticmethod
    def _s() -> int:
        return torch.cuda.current_stream().cuda_stream

    # ------------------------------------------------------------------ phases
    def publish(self) -> None:
        """set_worker_weights: the actors' copy of the online network (noise included)."""
        s = self._s()
        self.hip.copy_f32(self.actor_flat.data_ptr(), self.learner.flat.data_ptr(), self.learner.P, s)
        self.hip.copy_f32(self.actor_eps.data_ptr(), self.learner.eps.data_ptr(), self.learner.eps.numel(), s)

    def actor_step(self, half: int | None = None, into=None) -> None:
        """One acting step of all E envs.  ``half`` (overlap mode): write the transitions into
        staging half ``half`` instead of the ring (see :meth:`apply_staged`); ``into``: an
        ``AqlInsert`` of E rows (C = E) to write them to instead -- e.g. a central-topology
        actor rank's packet buffer (engine.central_aql); no tree write then."""
        h, s, E, r = self.hip, self._s(), self.E, self.replay
        if into is None and half is None and self._tail is not None:
            self._propose_q(h, s, E)
            h.aql_act_tail(self._tail, s)
            return
        self._act(h, s, E)
        if into is not None or half is not None:
            dst = into if into is not None else self._stage_ins[half]
            h.aql_env_step(self.env, self.env_act.data_ptr(), self.act_idx.data_ptr(), self.amu.data_ptr(), dst, s)
            self.actor_ctr.add_(1)  # the acting RNG counter (per_write_leaves bumps it otherwise)
            return
        h.aql_env_step(self.env, self.env_act.data_ptr(), self.act_idx.data_ptr(), self.amu.data_ptr(), self.ins, s)
        h.per_write_leaves(r.tree, self.slots.data_ptr(), 0, E, r.alpha, r.max_prio.data_ptr(), 0,
                           r.sorted_scratch.data_ptr(), r.filled.data_ptr(), E, self.actor_ctr.data_ptr(), 1, s)

    def _propose_q(self, h, s, E) -> None:
        """Proposal and candidate Q (the learner's MFMA candidate forward on the online net, s
        only) for all E envs."""
        # (the effective NoisyNet weights ride along in the proposal launch)
        h.aql_propose(self.actor_net, self.obs_buf.data_ptr(), E, self.low.data_ptr(), self.high.data_ptr(),
                      self.var.data_ptr(), self.seed ^ 0x9909, self.actor_ctr.data_ptr(), self.amu.data_ptr(), 0, s,
                      self.ws.data_ptr())
        h.aql_act_q(self.actL, s)

    def _act(self, h, s, E) -> None:
        """Proposal, candidate Q and epsilon-greedy selection for all E envs."""
        self._propose_q(h, s, E)
        h.aql_select(self.qbuf.data_ptr(), self.amu.data_ptr(), E, self.T, self.adim, self.eps.data_ptr(),
                     self.seed ^ 0xA9C1, self.actor_ctr.data_ptr(), self.act_idx.data_ptr(), self.env_act.data_ptr(), s)

    def apply_staged(self, half: int) -> None:
        """Overlap mode, learner stream: staging half ``half`` -> the ring at max priority."""
        h, s, E, r = self.hip, self._s(), self.E, self.replay
        h.aql_apply_staged(self._stage_ins[half], self.ins, E, self.obs, self.T * self.adim, s)
        h.per_write_leaves(r.tree, self.slots.data_ptr(), 0, E, r.alpha, r.max_prio.data_ptr(), 0,
                           r.sorted_scratch.data_ptr(), r.filled.data_ptr(), E, 0, 0, s)

    def learn_steps(self, publish: bool = False, gate: torch.Tensor | None = None) -> bool:
        """The iteration's K SGD steps; in the fused sequence each step but the last also draws
        the next step's rows (nothing inserts between them), so only the first forward samples.
        ``publish``: the last step also writes the acting copies (returns whether it did).
        ``gate``: only the first ``gate[0]`` of the K steps run (:meth:`AQLLearner.step`)."""
        pre = self.learner.predraw
        pub = False
        for k in range(self.K):
            pub = bool(self.learner.step(drawn=pre and k > 0, draw_next=pre and k + 1 < self.K,
                                         publish=publish and k + 1 == self.K, gate=gate, j=k))
        return pub

    def fill(self, threshold: int | None = None) -> None:
        """Act until the replay holds more than ``threshold`` transitions (AQL_dis.py:120:
        learning starts once len(buffer) > batch_size)."""
        thr = threshold if threshold is not None else (self.cfg.threshold or self.cfg.batch_size + 1)
        n = max(1, -(-int(thr) // self.E))
        if self.overlap:  # staged halves applied right away, plus one more left staged for the first iteration
            for i in range(n + 1):
                self.actor_step(self._half)
                if i < n:
                    self.apply_staged(self._half)
                self._half ^= 1
            self.publish()
            return
        for _ in range(n):
            self.actor_step()
        self.iterations = self._iterations  # (resyncs the fused tail's device iteration counter)
        self.publish()

    def capture(self) -> None:
        """The iteration (actor step + the K learner steps) as one hipGraph; overlap mode: one
        actor graph and one learner graph (apply + K steps) per staging half."""
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):  # warm the launch paths outside capture
            torch.cuda.synchronize(self.device)
        if self.overlap:
            self._g_actor, self._g_learn = [], []
            for hh in (0, 1):
                ga, gl = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(ga):
                    self.actor_step(hh)
                with torch.cuda.graph(gl):
                    self.apply_staged(1 - hh)
                    self.learn_steps()
                self._g_actor.append(ga)
                self._g_learn.append(gl)
            torch.cuda.synchronize(self.device)
            self._ev_learn.record(torch.cuda.current_stream(self.device))
            return
        # the whole serial iteration (acting + K steps) as ONE graph: one graph launch per
        # iteration instead of two (19.32-19.35k vs 19.10-19.13k SGD steps/s, one box)
        self._g_iter = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g_iter):
            self.actor_step()
            self._pub_in_graph = self.learn_steps(publish=True)
        torch.cuda.synchronize(self.device)

    def _beta(self) -> float:
        c = self.cfg  # AQL_dis.py:59 operator precedence kept
        return min(1.0, c.beta_start + self.iterations * (1.0 - c.beta_start) / c.max_step * c.n_workers)

    @property
    def iterations(self) -> int:
        return self._iterations

    @iterations.setter
    def iterations(self, v: int) -> None:
        """An assignment from outside the iteration loop (a checkpoint load, the central
        engine's recorded-batch count): the fused acting tail's device iteration counter, which
        computes the PER beta on the device (AQL_dis.py:59), follows it -- the two can never
        disagree silently.  The loop's own increments go to ``_iterations`` (the tail kernel
        bumps its device copy itself)."""
        self._iterations = int(v)
        if getattr(self, "_tail", None) is not None:
            self._iter_dev.fill_(self._iterations)

    def iteration(self) -> None:
        """One actor step of all envs, weight publish, K learner steps."""
        if self.overlap:
            return self._iteration_overlap()
        if self._tail is None:  # (the fused acting tail writes it on the device)
            self.learner.beta.fill_(self._beta())
        if self._g_iter is not None:
            self._g_iter.replay()
            pub = self._pub_in_graph
        else:
            self.actor_step()
            pub = self.learn_steps(publish=True)
        if not pub:
            self.publish()
        before = self.learner_steps
        self.learner_steps += self.K
        if target_sync_due(self.cfg, self.iterations, before, self.learner_steps):
            self.learner.sync_target()
            self.target_syncs.append(self.iterations)
        self._iterations += 1

    def _iteration_overlap(self) -> None:
        """Acting step t (staging half h) on the acting stream || the learner (apply half 1-h,
        the acting step t-1's, then K SGD steps) on the caller's stream.  Events: acting t
        waits for the learner t-1 (its publish); the learner t waits for acting t-1 (the half
        it applies) and, before publishing into the acting weights, for acting t."""
        hh = self._half
        L, A = torch.cuda.current_stream(self.device), self._astream
        A.wait_event(self._ev_learn)
        with torch.cuda.stream(A):
            if self._g_actor is not None:
                self._g_actor[hh].replay()
            else:
                self.actor_step(hh)
        self._ev_actor[hh].record(A)
        L.wait_event(self._ev_actor[1 - hh])
        self.learner.beta.fill_(self._beta())
        if self._g_learn is not None:
            self._g_learn[hh].replay()
        else:
            self.apply_staged(1 - hh)
            self.learn_steps()
        L.wait_event(self._ev_actor[hh])
        self.publish()
        before = self.learner_steps
        self.learner_steps += self.K
        if target_sync_due(self.cfg, self.iterations, before, self.learner_steps):
            self.learner.sync_target()
            self.target_syncs.append(self.iterations)
        self._iterations += 1
        self._ev_learn.record(L)
        self._half ^= 1

    def finished_episodes(self) -> list[tuple[float, int]]:
        """(return, length) of the episodes finished since the last call (host sync)."""
        n = int(self.ep_count.item())
        lo = max(self._ep_read, n - self.log_cap)
        out = []
        if n > lo:
            log = self.ep_log.cpu()
            out = [(float(log[k % self.log_cap, 0]), int(log[k % self.log_cap, 1])) for k in range(lo, n)]
        self._ep_read = n
        return out

    @property
    def transitions_per_iteration(self) -> int:
        return self.E
