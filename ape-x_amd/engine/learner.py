"""Fused, host-sync-free DQN learner step.

One learner step (reference: learner.py:152-175 + utils.py:64-97 + the replay
server's sample/update round trips over TCP) is, entirely on one HIP stream:

  per_sample (stratified PER, IS weights)  ->  gather s/s' u8 stacks from the frame ring
  -> Q(s) with grad, Q(s'), Q_target(s')   (fp32 MFMA trunk by default = the reference's
                                            precision; bf16-operand MFMA trunk opt-in)
  -> dqn_loss (double-DQN n-step Huber + IS weights + priorities + dL/dQ, one kernel)
  -> backward into ONE flat fp32 grad buffer  (-> optional RCCL all-reduce, DP)
  -> grad_sumsq + clip + centered RMSprop over the flat buffer (two kernels)
  -> priority write-back into the tree (leaf write + level recompute)

No ``.cpu()``/``.item()`` anywhere: priorities, indices, weights, loss and the grad
norms stay on device, so the step is capturable as a hipGraph and replayed.
The model keeps the reference state_dict (parameters are views of the flat buffer).
"""
from __future__ import annotations

import copy
from dataclasses import dataclass
from types import SimpleNamespace

import torch

from .. import ops
from ..models.dqn import DuelingDQN
from ..models.fused import DTYPES, forward_multi, make_hip_net, make_workspace
from .hbm_replay import HBMReplay


@dataclass
class LearnerConfig:
    batch_size: int = 512
    n_step: int = 3
    gamma: float = 0.99
    lr: float = 6.25e-5
    rms_alpha: float = 0.95
    rms_eps: float = 1.5e-7
    centered: bool = True
    max_norm: float = 40.0
    lr_gamma: float = 1.0          # StepLR gamma (ApeX.py: 0.99 every 1000 steps)
    lr_step_size: int = 0
    lr_step_offset: int = 0
    beta: float = 0.4
    optimizer: str = "rmsprop"     # or "adam"
    forward: str = "torch"         # "torch" (PyTorch/MIOpen modules) | "hip" (hand-written MFMA kernels)
    dtype: str = "fp32"            # compute precision: "fp32" (reference, learner.py:139-145: fp32 MFMA on the
                                   # hip path, no autocast on the torch path) | "bf16" (opt-in fast mode)
    seed: int = 0
    # the sampling launch copies every sampled row (frame ids, action, return, done) into
    # private buffers that the forward, loss and backward read: writers of the replay tables
    # may then run beside the step (the central topology's ingest, engine/central.py)
    private_rows: bool = False
    # the step's priority-tree write as extra workgroups of the trunk backward's launches (the
    # leaves with the FC1 pair, level 1 with the conv3 pair, level 2 + the top with the conv2
    # pair: ops/csrc/tree_dev.h tree_ride) instead of a forked tree stream joined before the
    # optimizer -- fp32 HIP learner, single process, no ingest tail
    tree_ride: bool = True
    # the PER draw folded into the fp32 conv1 forward launch (every workgroup draws its own
    # samples; f32_conv1_fwd_x3_k) instead of its own sampling launch at the chain head --
    # single replay, no private rows
    draw_in_conv1: bool = True


def forward_q(model: DuelingDQN, x_u8: torch.Tensor, bf16: bool = False) -> torch.Tensor:
    """Q = V + A - mean(A) in fp32 (the reference feeds raw 0..255 values);
    ``bf16``: the conv trunk under bf16 autocast (u8 frames are exact in bf16), fp32 heads."""
    if bf16:
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            h = model.features(x_u8.to(torch.bfloat16))
        h = h.float().flatten(1)
    else:
        h = model.features(x_u8.float()).flatten(1)
    adv = model.advantage(h)
    val = model.value(h)
    return val + adv - adv.mean(1, keepdim=True)


class DQNLearner:
    BLOCKS_PER_SEG = 16

    def __init__(self, model: DuelingDQN, replay: HBMReplay, cfg: LearnerConfig, allreduce=None, sharded=None):
        self.hip = ops.hip()
        self.cfg = cfg
        if cfg.dtype not in DTYPES:
            raise ValueError(f"LearnerConfig.dtype must be one of {DTYPES}, got {cfg.dtype!r}")
        self.fp32 = cfg.dtype == "fp32"
        self.replay = replay
        self.device = replay.device
        self.model = model.to(self.device)
        self.flat = self.model.flatten_parameters()
        self.target = copy.deepcopy(self.model)
        self.target._flat = None
        self.tflat = self.target.flatten_parameters()
        for p in self.target.parameters():
            p.requires_grad_(False)
        self.P = self.flat.numel()
        dev = self.device
        # gradient buffer = [shard slots (sharded DP) + padding | flat gradient]: the slots
        # ride the conv-gradient all-reduce (parallel.sharded); the padding keeps the flat
        # gradient 256-byte aligned
        self.dp_split_possible = allreduce is not None and cfg.forward == "hip"
        ns = 2 * sharded.world if (sharded is not None and self.dp_split_possible) else 0
        self.grad_prefix = -(-ns // 64) * 64
        self.grad_buf = torch.zeros(self.grad_prefix + self.P, dtype=torch.float32, device=dev)
        self.flat_grad = self.grad_buf[self.grad_prefix:]
        if ns:
            sharded.slots = self.grad_buf[:ns]
        off = 0
        for p in self.model.parameters():
            n = p.numel()
            p.grad = self.flat_grad[off:off + n].view_as(p)
            off += n
        self.segments = self.model.param_segments()
        self.partials = torch.zeros(self.hip.grad_norm_partials(), dtype=torch.float64, device=dev)
        self.opt_s1 = torch.zeros(self.P, dtype=torch.float32, device=dev)
        self.opt_s2 = torch.zeros(self.P, dtype=torch.float32, device=dev)
        if cfg.optimizer == "rmsprop":
            self.hp = self.hip.RMSpropParams(cfg.lr, cfg.rms_alpha, cfg.rms_eps, cfg.max_norm, cfg.lr_gamma,
                                             cfg.lr_step_size, cfg.lr_step_offset, cfg.centered)
        elif cfg.optimizer == "adam":
            self.hp = self.hip.AdamParams(cfg.lr, max_norm=cfg.max_norm, lr_gamma=cfg.lr_gamma,
                                          lr_step_size=cfg.lr_step_size, lr_step_offset=cfg.lr_step_offset)
        else:
            raise ValueError(cfg.optimizer)
        B, A = cfg.batch_size, self.model.num_actions
        self.B, self.A = B, A
        self.idx = torch.zeros(B, dtype=torch.int32, device=dev)
        self.w = torch.zeros(B, dtype=torch.float32, device=dev)
        self.s = torch.zeros(B, 4, 84, 84, dtype=torch.uint8, device=dev)
        self.s2 = torch.zeros_like(self.s)
        self.a = torch.zeros(B, dtype=torch.int32, device=dev)
        self.r = torch.zeros(B, dtype=torch.float32, device=dev)
        self.d = torch.zeros(B, dtype=torch.float32, device=dev)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self.dq = torch.zeros(B, A, dtype=torch.float32, device=dev)
        self.prio = torch.zeros(B, dtype=torch.float32, device=dev)
        self.norms = torch.zeros(4, dtype=torch.float32, device=dev)   # l2, (unused), clip coef, lr
        self.step_counter = torch.zeros(1, dtype=torch.int64, device=dev)
        self.beta = torch.full((1,), cfg.beta, dtype=torch.float32, device=dev)
        self.gamma_n = float(cfg.gamma ** cfg.n_step)
        # data-parallel learners: parallel.dp.FlatGradAllReduce (async SUM; the optimizer
        # applies the 1/world mean through grad_scale)
        self.allreduce = allreduce
        if allreduce is not None:
            self.hp.grad_scale = 1.0 / allreduce.world
        self.sharded = sharded      # parallel.sharded.ShardedSampling (global PER over shards)
        self.host_steps = 0
        self.hip_net = cfg.forward == "hip"
        self.n_fin_partials = 0
        if self.hip_net:
            self.net = make_hip_net(self.model, cfg.dtype)
            self.net.enable_backward(B)
            self.tnet = make_hip_net(self.target, cfg.dtype)
            # the optimizer refreshes the packed weight copies (bf16 or exact fp32) in its pass
            self.pmap1, self.pmap2 = self.net.pack_maps()
            self.ws_s = make_workspace(B, A, dev, cfg.dtype, keep_for_backward=True)
            self.ws_s2 = make_workspace(B, A, dev, cfg.dtype)
            self.ws_t = make_workspace(B, A, dev, cfg.dtype)
            # fused loss + heads backward (dqn_heads_bwd) outputs; the priority-tree write
            # (which mixes the TD errors into priorities and forms the loss mean) runs on
            # a forked stream concurrently with the trunk backward
            self.delta = torch.zeros(B, dtype=torch.float32, device=dev)
            self.lw = torch.zeros(B, dtype=torch.float32, device=dev)
            self.lh_blocks = self.hip.dqn_heads_bwd_blocks(B)
            self.lh_part = torch.zeros(self.lh_blocks * ((A + 1) * 128 + (A + 1) + 256), dtype=torch.float32,
                                       device=dev)
            self.step_snap = torch.zeros(1, dtype=torch.int64, device=dev)
            # (a high-priority tree stream -- its single-workgroup kernels otherwise wait for CU
            # room beside the backward -- measured 1011 vs 2492 learner steps/s: not used)
            self.tree_stream = torch.cuda.Stream(device=dev)
            # single-process learner: grad_finalize writes the grad-norm partials (every
            # gradient passes through it), so no separate sum-of-squares pass; with an
            # all-reduce the norm must be taken after it (grad_sumsq)
            self.fin_partials = torch.zeros(8192, dtype=torch.float64, device=dev)
            self.n_fin_partials = 0
        self._src = None  # (s ids, s' ids, idx, transition table) of the batch in flight
        self.rows = replay.row_buffers(B) if cfg.private_rows else None
        # one-shot callables run on the tree stream AFTER this step's priority write (the
        # central engine's ingest: its leaf writes must follow the learner's for a shared slot)
        self.tree_tail = []
        # one-shot callables run on the tree stream before this step's priority write
        # (the overlapped engine's deferred actor-row priorities)
        self.tree_hooks = []
        # staged actor rows whose priorities go into this step's batched tree write:
        # (slots, raw priorities, counter advanced by the row count)
        self.pre_writes = []
        # staged actor rows scattered into the tables by the sampling launch:
        # (staged table ptr dict, slots, raw priorities)
        self.pre_rows = []
        self.tree_rides_used = False  # the last traced trunk backward carried the tree riders
        self.draws_in_conv1 = False   # the last traced forward drew its batch inside conv1

    @staticmethod
    def _stream() -> int:
        return torch.cuda.current_stream().cuda_stream

    # ------------------------------------------------------------------ phases
    @property
    def dp_split(self) -> bool:
        """Data-parallel HIP learner: the backward runs as two phases so the FC1/head
        gradients (the tail of the flat buffer, ~91% of its bytes) are all-reduced while
        the conv backward runs (:meth:`forward_phase` / :meth:`backward_phase`)."""
        return self.dp_split_possible

    def grad_slices(self) -> tuple[torch.Tensor, torch.Tensor]:
        """(FC1 + heads tail, [shard slots +] conv head) views of the gradient buffer, in
        all-reduce order."""
        fc_off = self.fc_grad_offset
        return self.flat_grad[fc_off:], self.grad_buf[:self.grad_prefix + fc_off]

    @property
    def fc_grad_offset(self) -> int:
        seg = {name: (o, n) for name, o, n in self.segments}
        off = seg["advantage.0.weight"][0]
        assert all((o + n <= off) == name.startswith("features.") for name, (o, n) in seg.items()), \
            "flat layout: conv parameters first, then the dueling heads"
        return off

    def sample_and_forward(self) -> None:
        """Sample, gather, forward x3, loss, backward (grads in ``flat_grad``)."""
        self.forward_phase()
        if self.dp_split:
            self.backward_phase()

    def forward_phase(self, part: str | None = None) -> None:
        """Sample, forward x3, loss + heads backward; single-process: the whole backward
        too; data-parallel split: up to the FC1 backward and its finalize.
        ``part`` (single-process HIP learner): "a" = up to the fused loss + heads backward,
        "b" = the trunk backward (+ the priority-tree branch) -- the two halves of the step
        around the point where the overlapped engine may start its actor graph."""
        if part == "b":
            self._trunk_phase()
            return
        s = self._stream()
        rp = self.replay
        glob = shard = None
        if self.sharded is not None:  # gathered shard masses -> global pmin + weight scale
            if self.sharded.in_kernel:
                shard = self.sharded.sample_args()
            else:
                self.sharded.finalize()
                glob = self.sharded.glob
        rows, self.pre_rows = self.pre_rows, []
        for extra in rows[:-1]:  # more than one staged actor step per learner step
            self.hip.apply_staged_rows(extra[0], self.replay.trans_ptrs(), extra[1].data_ptr(), extra[2].data_ptr(),
                                       extra[1].numel(), s)
        draw = self._conv1_draw(rows[-1] if rows else None) if glob is None and shard is None else None
        self.draws_in_conv1 = draw is not None
        if draw is None:
            self.replay.sample_indices(self.B, self.idx, self.w, self.step_counter, self.beta, glob=glob,
                                       shard=shard, rows=rows[-1] if rows else None, out_rows=self.rows)
        if self.rows is not None:  # the batch reads its private rows (no idx indirection)
            self._src = (self.rows["s_ids"], self.rows["s2_ids"], None, SimpleNamespace(**self.rows))
        else:
            self._src = (rp.s_ids, rp.s2_ids, self.idx, rp)
        self._forward_and_loss(s, part, draw)

    def _conv1_draw(self, rows):
        """The PER draw (+ the staged actor rows ``rows`` it scatters) as part of the conv1
        forward launch -- the slots, IS weights and rows per_sample writes -- or None when the
        draw keeps its own launch (no fp32 HIP forward, private rows)."""
        rp = self.replay
        if not (self.cfg.draw_in_conv1 and self.hip_net and self.fp32 and self.rows is None):
            return None
        st = {} if rows is None else {"rows_stage": rows[0], "rows_dst": rp.trans_ptrs(),
                                      "rows_slot": rows[1].data_ptr(), "rows_prio": rows[2].data_ptr(),
                                      "rows_E": rows[1].numel()}
        return self.hip.make_conv_sample(rp.tree, rp.filled.data_ptr(), self.beta.data_ptr(), rp.seed,
                                         self.step_counter.data_ptr(), self.idx.data_ptr(), self.w.data_ptr(),
                                         int(not rp.exact_mass), **st)

    def _forward_and_loss(self, s: int, part: str | None = None, draw=None) -> None:
        """Forward x3 + loss (+ the backward: single process) of the batch in ``_src``
        (``draw``: the PER draw folded into the conv1 launch)."""
        rp = self.replay
        if self.hip_net:
            # conv1 reads the sampled stacks straight out of the HBM frame ring (no gather),
            # the loss reads (a, r, d) straight out of the transition table.  The three passes
            # share each layer's launch (5 kernels, not 15).
            ids_s, ids_s2, jdx, tab = self._src
            forward_multi([(self.net, rp.frames, self.ws_s, ids_s, jdx), (self.net, rp.frames, self.ws_s2, ids_s2, jdx),
                           (self.tnet, rp.frames, self.ws_t, ids_s2, jdx)], draw=draw)
            q2t = self.ws_t.q
            m = self.model
            self.hip.dqn_heads_bwd(
                {"q": self.ws_s.q.data_ptr(), "q2": self.ws_s2.q.data_ptr(), "q2t": q2t.data_ptr(),
                 "act": tab.action.data_ptr(), "rew": tab.reward.data_ptr(), "done": tab.done.data_ptr(),
                 "idx": 0 if jdx is None else jdx.data_ptr(), "w": self.w.data_ptr(), "h": self.ws_s.h.data_ptr(),
                 "w_adv2": m.advantage[2].weight.data_ptr(), "w_val2": m.value[2].weight.data_ptr(),
                 "delta": self.delta.data_ptr(), "lw": self.lw.data_ptr(),
                 ("dz" if self.fp32 else "dz_bf"): (self.ws_s.dz if self.fp32 else self.ws_s.dz_bf).data_ptr(),
                 "part": self.lh_part.data_ptr(), "step": self.step_counter.data_ptr(),
                 "step_snap": self.step_snap.data_ptr(),
                 **({"dzx": self.ws_s.dzx.data_ptr(), "dzx_ps": self.ws_s.dzx.shape[1]}
                    if getattr(self.ws_s, "dzx", None) is not None else {})}, self.B, self.A, self.gamma_n, s)
            if self.dp_split:
                heads_job = self.net.heads_finalize_job(self.lh_part, self.lh_blocks)
                self.net.fc_backward(self.ws_s, extra_jobs=[heads_job])
                return
            if part != "a":
                self._trunk_phase()
            return
        assert draw is None, "the folded draw needs the HIP forward"
        hooks, self.tree_hooks = self.tree_hooks, []
        for fn in hooks:  # no tree stream on this path: deferred priorities go right after sampling
            fn()
        self.replay.gather(self.idx, self.s, self.s2, self.a, self.r, self.d)
        bf = not self.fp32
        q = forward_q(self.model, self.s, bf)
        with torch.no_grad():
            q2 = forward_q(self.model, self.s2, bf)
            q2t = forward_q(self.target, self.s2, bf)
        q2 = q2.contiguous()
        q2t = q2t.contiguous()
        qd = q.detach().contiguous()
        self.hip.dqn_loss(qd.data_ptr(), q2.data_ptr(), q2t.data_ptr(), self.A, self.a.data_ptr(), self.r.data_ptr(),
                          self.d.data_ptr(), 0, self.w.data_ptr(), self.B, self.A, self.gamma_n, self.loss.data_ptr(),
                          self.dq.data_ptr(), self.prio.data_ptr(), s)
        self.flat_grad.zero_()
        q.backward(self.dq)

    def _trunk_phase(self) -> None:
        """Single-process HIP learner: FC1 + conv backward and the finalize (the heads'
        partials folded in), the priority-tree branch forked beside it and joined at the end."""
        assert self.hip_net and not self.dp_split
        rp = self.replay
        ids_s, _, jdx, _ = self._src
        heads_job = self.net.heads_finalize_job(self.lh_part, self.lh_blocks)
        sumsq = self.fin_partials if self.allreduce is None else None
        rides = self._tree_rides()
        self.tree_rides_used = rides is not None
        if rides is not None:  # the tree write rides the backward launches: no fork / join
            n = self.net.trunk_backward(rp.frames, self.ws_s, ids_s, jdx, extra_jobs=[heads_job], sumsq=sumsq,
                                        rides=rides)
        else:
            after = self._fork_point()
            n = self.net.trunk_backward(rp.frames, self.ws_s, ids_s, jdx, extra_jobs=[heads_job], sumsq=sumsq,
                                        after_first=after)
        if self.allreduce is None:
            assert n <= self.fin_partials.numel()
            self.n_fin_partials = n
        if rides is None:
            self._tree_fork_end()

    def _tree_rides(self):
        """Riders of this step's tree write for the FC1, conv3 and conv2 backward launches and the
        gradient finalize (leaves, level 1, level 2 or the top walk, the top walk or None) -- the staged actor
        rows' priorities then the learner's mixed, deduplicated priorities, the same leaves,
        nodes, max priority and counters as :meth:`tree_phase` -- or None when the write keeps
        the forked tree stream (no fp32 HIP trunk, hooks / an ingest tail queued, several staged
        actor writes, or a tree too tall for two wide levels)."""
        rp = self.replay
        if not (self.cfg.tree_ride and self.fp32 and hasattr(self.net, "fc1_ride_ok") and not self.tree_hooks
                and not self.tree_tail and len(self.pre_writes) <= 1):
            return None
        stages = self.hip.tree_ride_level_stages(rp.tree)
        pre = self.pre_writes[0] if self.pre_writes else None
        E = 0 if pre is None else pre[0].numel()
        if stages < 0 or E + self.B > rp.wlist.numel():
            return None
        self.pre_writes = []
        ptr = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
        common = (ptr(pre[0]) if pre else 0, ptr(pre[1]) if pre else 0, E, ptr(pre[2]) if pre else 0,
                  self.idx.data_ptr(), self.B, self.delta.data_ptr(), self.lw.data_ptr(), self.prio.data_ptr(),
                  self.loss.data_ptr(), self.step_counter.data_ptr(), rp.owner.data_ptr(), rp.wlist.data_ptr(),
                  rp.max_prio.data_ptr(), rp.alpha)
        L = rp.tree.levels
        mk = self.hip.make_tree_ride
        leaves, lv1 = mk(rp.tree, 1, 0, 0, *common), mk(rp.tree, 2, 1, 0, *common)
        if stages == 1:  # the top walk (levels 2..) with the conv2 pair
            return leaves, lv1, (mk(rp.tree, 3, 0, 2, *common) if L >= 2 else None), None
        # level 2 with the conv2 pair, the top walk (levels 3..) with the gradient finalize (as
        # block 0 of the conv1 weight gradient's 256 one-per-CU workgroups it pushed the last
        # of them into a second round: +1.8 us)
        return leaves, lv1, mk(rp.tree, 2, 2, 0, *common), mk(rp.tree, 3, 0, 3, *common)

    def backward_phase(self, after_first=None) -> None:
        """Data-parallel split, part 2: priority-tree writes on the forked tree stream beside
        the conv backward (+ its finalize); joined before returning."""
        assert self.dp_split
        rp = self.replay
        tree = self._fork_point()
        after = tree if after_first is None else (lambda: (tree(), after_first()))
        ids_s, _, jdx, _ = self._src
        self.net.conv_backward(rp.frames, self.ws_s, ids_s, jdx, after_first=after)
        self._tree_fork_end()
        if self.sharded is not None and self.grad_prefix:
            # the tree is final for the next sample: pack this shard's slot, which the
            # conv-gradient all-reduce then exchanges (the next step's shard masses)
            self.sharded.pack()

    def _fork_point(self):
        """Fork the tree branch HERE (it depends on everything launched so far) but capture
        it after the backward's first launch: in the captured graph the backward chain is
        then the first child of the fork and keeps the launch queue, and only the tree
        branch pays the cross-queue hand-off.  Returns the callback for ``after_first``."""
        self._ev_fork = ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        return lambda: self._tree_fork_begin(ev)

    def _tree_fork_begin(self, ev: torch.cuda.Event) -> None:
        """Fork: deferred actor-row priorities, then the priority mix + loss mean + tree
        write (+ step bump) of this step's samples, on the tree stream beside the backward
        (``ev``: the fork point, recorded earlier on the main stream).  The tree write is
        the single-workgroup level walk: it occupies few CUs beside the backward GEMMs."""
        self.tree_stream.wait_event(ev)
        with torch.cuda.stream(self.tree_stream):
            self.tree_phase()

    def tree_phase(self) -> None:
        """The priority-tree work of this step on the CURRENT stream (the forked branch's body)."""
        hooks, self.tree_hooks = self.tree_hooks, []
        for fn in hooks:
            fn()
        pre, self.pre_writes = self.pre_writes, []
        for slots, prios, filled in pre:
            self.replay.write_priorities(slots, prios, dedup=False, bumps=((filled, slots.numel()),))
        # the single-workgroup walks (rank-sorted dedup, one workgroup per walk) on purpose:
        # the batched per_write_batch (one wide launch per big tree level) finishes sooner
        # but its workgroups compete with the backward GEMMs beside it -- measured 2188 vs
        # 2303 learner steps/s (MI355X, round 5, interleaved; profiles/r5_x6.md)
        self.replay.write_priorities(self.idx, None, dedup=True, bumps=((self.step_counter, 1),),
                                     mix=(self.delta, self.lw, self.prio, self.loss))
        tail, self.tree_tail = self.tree_tail, []
        for fn in tail:
            fn()

    def _tree_fork_end(self) -> None:
        torch.cuda.current_stream().wait_stream(self.tree_stream)  # join: the next sample reads the tree

    def optimize(self) -> None:
        s = self._stream()
        h = self.hip
        if self.hip_net and self.n_fin_partials:
            parts, nparts = self.fin_partials, self.n_fin_partials  # from grad_finalize
        else:
            h.grad_sumsq(self.flat_grad.data_ptr(), self.P, self.partials.data_ptr(), s)
            parts, nparts = self.partials, self.partials.numel()
        if not self.hip_net:
            pk = {}
        elif self.fp32:  # exact fp32 packed copies (PackMap.arena_f32 + FC1 tiles)
            pk = self.net.opt_pack_args()
        else:  # bf16 packed copies
            pk = {"dst1": self.pmap1.data_ptr(), "dst2": self.pmap2.data_ptr(), "arena": self.net.arena.data_ptr(),
                  **self.net.fc_pack_args()}
        step = h.rmsprop_step if self.cfg.optimizer == "rmsprop" else h.adam_step
        # the fused path already bumped step_counter on the tree stream: the optimizer reads
        # this step's snapshot instead
        stp = self.step_snap if self.hip_net else self.step_counter
        step(self.flat.data_ptr(), self.flat_grad.data_ptr(), self.opt_s1.data_ptr(), self.opt_s2.data_ptr(), self.P,
             parts.data_ptr(), nparts, self.hp, stp.data_ptr(), self.norms.data_ptr(), s, **pk)
        if not self.hip_net:
            self.replay.write_priorities(self.idx, self.prio, dedup=True, bumps=((self.step_counter, 1),))

    def step(self) -> None:
        """One eager learner step (the engine runs the same phases as hipGraphs)."""
        if self.sharded is not None:
            self.sharded.exchange()
        self.forward_phase()
        if self.allreduce is None:
            pass
        elif self.dp_split:
            fc, conv = self.grad_slices()
            w1 = self.allreduce.start(fc)
            self.backward_phase()
            w2 = self.allreduce.start(conv)
            self.allreduce.wait(w1, w2)
        else:
            self.allreduce.wait(self.allreduce.start(self.flat_grad))
        self.optimize()
        self.host_steps += 1

    # ------------------------------------------------------------------ target / params
    def refresh_packed(self) -> None:
        """Re-derive the packed weight copies from the fp32 master (after the flat buffer
        was written outside the optimizer, e.g. a DP broadcast or a checkpoint load)."""
        if self.hip_net:
            self.net.repack()

    def sync_target(self) -> None:
        self.hip.copy_f32(self.tflat.data_ptr(), self.flat.data_ptr(), self.P, self._stream())
        if self.hip_net:
            self.tnet.copy_packed_from(self.net)

    def copy_params_to(self, dst_flat: torch.Tensor) -> None:
        self.hip.copy_f32(dst_flat.data_ptr(), self.flat.data_ptr(), self.P, self._stream())

    def state_dict(self):
        return self.model.state_dict()

    def stats(self) -> dict:
        """Host-side view of the last step's scalars (forces a sync; call rarely).
        ``grad_norm`` is the reference's logged value (sum_p ||g_p||^(1/2))^(1/2) of the last
        step's (pre-clip) gradient, ``grad_norm_l2`` the true global L2 used for clipping."""
        n = self.norms.tolist()
        # under data parallelism flat_grad holds the all-reduced SUM; the optimizer applies
        # the 1/world mean (grad_scale) in-kernel, so scale the logged norm the same way
        sc = float(self.hp.grad_scale) if self.allreduce is not None else 1.0
        ref = sum((sc * self.flat_grad[o:o + k].norm().item()) ** 0.5 for _, o, k in self.segments) ** 0.5
        return {"loss": float(self.loss.item()), "grad_norm_l2": n[0], "grad_norm": ref, "clip": n[2], "lr": n[3]}
