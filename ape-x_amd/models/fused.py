"""HIP fast path of the dueling Q-network (forward on hand-written MFMA kernels).

``HipDuelingNet`` wraps a :class:`DuelingDQN` (fp32 master parameters, reference
state_dict, flat buffer) and keeps a packed bf16 copy of its weights in the layouts the
gfx950 kernels want (conv weights [N][KH][KW][C] and their transposes for dgrad, FC1
repacked to the channels-last flatten order), all in one bf16 arena.  The learner's
fused optimizer rewrites the arena in the same pass as the fp32 update (``pack_maps``
-> PackMap), target sync / actor publish copy arenas, and ``repack()`` re-derives it
from scratch (init, after a broadcast or checkpoint load).

Forward (per pass, no autograd):
  conv_fwd x3  (u8 frames -> bf16 NHWC activations; MFMA 32x32x16, bias+ReLU fused)
  (``forward_multi``: up to 3 passes share each launch -- 5 kernels for the learner's
  Q(s), Q(s'), Q_target(s'))
  fc1_fwd      (split-K MFMA GEMM, 128-row x 256-column tiles with the W slice staged
               once in LDS, 14-28 fp32 partial slabs; bytes per CU, not grid size, bound
               this skinny K = 3136 shape)
  heads_fwd    (partial sum + bias + ReLU + adv/value heads + dueling combine, one wave per row)
Backward (explicit, writes every parameter gradient into the flat fp32 grad buffer
exactly once, so no zeroing pass is needed; the learner fuses the loss and heads part
into one launch, ``dqn_heads_bwd``, and all batch-sliced reductions into one
``grad_finalize``):
  heads_bwd -> head weight/bias grads (small GEMMs/sums) -> FC1 dW/dX (fc1_bwd_k MFMA) ->
  conv3/conv2/conv1: MFMA wgrad (ds_read_b64_tr_b16 operand transposes, split over the
  batch, deterministic partial reduce, conv bias grads fused) and MFMA dgrad (stride-1
  zero-border / stride-2 sub-pixel implicit GEMM with the ReLU backward fused).

Numerics: bf16 operands, fp32 accumulation, fp32 heads and Q.  Checked against the
fp32 PyTorch module in tests/test_gpu_fused_net.py.  This is the opt-in ``dtype="bf16"``
mode; the reference-precision default is ``fused_f32.F32DuelingNet`` (fp32 MFMA).
"""
from __future__ import annotations

import torch

from .. import ops
from .dqn import DuelingDQN

P3, C3 = 49, 64
FEAT = P3 * C3  # 3136
FC1_SPLITS = 28  # max split-K slabs an FC1 launch writes (fc_kernels.hip fc1_splits())


class NetWorkspace:
    """Activation buffers for one forward pass of batch ``B``."""

    def __init__(self, B: int, A: int, device, keep_for_backward: bool = False):
        self.B, self.A = B, A
        bf = dict(dtype=torch.bfloat16, device=device)
        f32 = dict(dtype=torch.float32, device=device)
        self.a1 = torch.empty(B, 400, 32, **bf)
        self.a2 = torch.empty(B, 81, 64, **bf)
        self.a3 = torch.empty(B, FEAT, **bf)
        self.z = torch.empty(FC1_SPLITS, B, 256, **f32)  # FC1 split-K partial slabs
        self.h = torch.empty(B, 256, **f32) if keep_for_backward else None
        self.q = torch.empty(B, A, **f32)
        if keep_for_backward:
            self.dA = torch.empty(B, A + 1, **f32)
            self.dz = torch.empty(B, 256, **f32)
            self.dz_bf = torch.empty(B, 256, **bf)
            self.da3 = torch.empty(B, FEAT, **bf)
            self.dy3 = torch.empty(B, P3, C3, **bf)
            self.dy2 = torch.empty(B, 81, 64, **bf)
            self.dy1 = torch.empty(B, 400, 32, **bf)


def _cl_view(t: torch.Tensor, B: int, C: int, H: int, W: int) -> torch.Tensor:
    """[B][H][W][C] memory viewed as a channels-last [B, C, H, W] tensor."""
    return t.as_strided((B, C, H, W), (H * W * C, 1, W * C, C))


class HipDuelingNet:
    fp32 = False
    # packed bf16 weights live in one arena: [w1p | w2p | w3p | wfc1p | w2t | w3t]
    # (conv1 keeps the reference layout [n][c][ky][kx]: its kernel's K order is (c, ky, kx))
    LAYOUT = (("w1p", (32, 4, 8, 8)), ("w2p", (64, 4, 4, 32)), ("w3p", (64, 3, 3, 64)), ("wfc1p", (256, FEAT)),
              ("w2t", (4, 4, 32, 64)), ("w3t", (3, 3, 64, 64)), ("wfc1t", (FEAT, 256)))

    def __init__(self, model: DuelingDQN):
        assert model.cnn and tuple(model.input_shape) == (4, 84, 84), "HIP path is the Atari Nature-CNN"
        self.hip = ops.hip()
        assert self.hip.fc1_splits() <= FC1_SPLITS, "fc_kernels.hip writes more split-K slabs"
        self.model = model
        self.A = model.num_actions
        dev = next(model.parameters()).device
        self.device = dev
        sizes = [int(torch.Size(sh).numel()) for _, sh in self.LAYOUT]
        self.arena = torch.empty(sum(sizes), dtype=torch.bfloat16, device=dev)
        self.arena_offsets = {}
        off = 0
        for (name, sh), n in zip(self.LAYOUT, sizes):
            setattr(self, name, self.arena[off:off + n].view(sh))
            self.arena_offsets[name] = off
            off += n
        self.fwd_numel = self.arena_offsets["w2t"]   # forward-only part of the arena
        self._wgrad_ws = None
        self._maps = None
        f = model.features
        self.b1, self.b2, self.b3 = f[0].bias, f[2].bias, f[4].bias
        self.repack()

    def pack_maps(self) -> tuple[torch.Tensor, torch.Tensor]:
        """int32 (dst1, dst2) over the model's flat parameter order: the arena positions
        that hold bf16 copies of each parameter (-1 = not packed, e.g. biases and the
        fp32 head weights).  Used by the fused optimizer (PackMap)."""
        if self._maps is not None:
            return self._maps
        m, f = self.model, self.model.features
        seg = {name: (o, n) for name, o, n in m.param_segments()}
        P = sum(n for _, n in seg.values())
        dst1 = torch.full((P,), -1, dtype=torch.int64)
        dst2 = torch.full((P,), -1, dtype=torch.int64)
        ao = self.arena_offsets

        def place(dst, pname, ref_of_pos, base):
            o, n = seg[pname]
            assert ref_of_pos.numel() == n
            dst[o + ref_of_pos] = base + torch.arange(n)

        for li, pname, N, C, K in ((0, "features.0.weight", 32, 4, 8), (1, "features.2.weight", 64, 32, 4),
                                   (2, "features.4.weight", 64, 64, 3)):
            ref = torch.arange(N * C * K * K).view(N, C, K, K)
            order = ref.reshape(-1) if li == 0 else ref.permute(0, 2, 3, 1).reshape(-1)
            place(dst1, pname, order, ao[("w1p", "w2p", "w3p")[li]])
            if li > 0:
                place(dst2, pname, ref.permute(2, 3, 1, 0).reshape(-1), ao[("w2t", "w3t")[li - 1]])
        ref = torch.arange(128 * FEAT).view(128, C3, P3).permute(0, 2, 1).reshape(-1)
        place(dst1, "advantage.0.weight", ref, ao["wfc1p"])
        place(dst1, "value.0.weight", ref, ao["wfc1p"] + 128 * FEAT)
        # W^T [k = p*64 + c][n] for the FC1 input-gradient GEMM (value rows at n + 128):
        # reference element (n, c*49 + p) -> wfc1t[(p*64 + c)*256 + n]
        n_i = torch.arange(128).view(128, 1, 1)
        c_i = torch.arange(C3).view(1, C3, 1)
        p_i = torch.arange(P3).view(1, 1, P3)
        post = ((p_i * C3 + c_i) * 256 + n_i).reshape(-1)  # in reference (n, c, p) order
        for pname, n0 in (("advantage.0.weight", 0), ("value.0.weight", 128)):
            o, n = seg[pname]
            dst2[o:o + n] = ao["wfc1t"] + n0 + post
        self._maps = (dst1.to(torch.int32).to(self.device), dst2.to(torch.int32).to(self.device))
        return self._maps

    def fc_pack_args(self) -> dict:
        """Keyword arguments of the fused optimizer's FC1 tile path (FcPack): the flat
        offsets of both FC1 weights and the two packed layouts they refresh."""
        seg = {name: o for name, o, _ in self.model.param_segments()}
        return {"fc_off0": seg["advantage.0.weight"], "fc_off1": seg["value.0.weight"],
                "fc_wp": self.wfc1p.data_ptr(), "fc_wt": self.wfc1t.data_ptr()}

    def copy_packed_from(self, other: "HipDuelingNet", forward_only: bool = True) -> None:
        """Device copy of another net's packed weights (same architecture)."""
        n = self.fwd_numel if forward_only else self.arena.numel()
        self.arena[:n].copy_(other.arena[:n])

    @staticmethod
    def _s() -> int:
        return torch.cuda.current_stream().cuda_stream

    def repack(self) -> None:
        h, s, f, m = self.hip, self._s(), self.model.features, self.model
        self.w1p.copy_(f[0].weight.detach().reshape(self.w1p.shape))  # bf16 cast, reference layout
        h.pack_conv_w(f[2].weight.data_ptr(), self.w2p.data_ptr(), 64, 32, 4, 4, s)
        h.pack_conv_w(f[4].weight.data_ptr(), self.w3p.data_ptr(), 64, 64, 3, 3, s)
        h.pack_fc1(m.advantage[0].weight.data_ptr(), m.value[0].weight.data_ptr(), self.wfc1p.data_ptr(), P3, C3, s)
        if self._wgrad_ws is not None:  # the backward is only used by the learner's online net
            h.pack_conv_wt(f[2].weight.data_ptr(), self.w2t.data_ptr(), 64, 32, 4, 4, s)
            h.pack_conv_wt(f[4].weight.data_ptr(), self.w3t.data_ptr(), 64, 64, 3, 3, s)
            self.wfc1t.copy_(self.wfc1p.t())

    def enable_backward(self, B: int | None = None) -> None:
        """Allocate backward workspaces + transposed weights (call before graph capture;
        ``B`` is unused: the bf16 workspaces are sized for any batch).
        One wgrad partial workspace per conv layer: the three layers' partials are reduced
        together by one grad_finalize launch at the end of the backward."""
        self._wgrad_wss = [torch.empty(self.hip.wgrad_workspace_floats(k), dtype=torch.float32, device=self.device)
                           for k in (1, 2, 3)]
        self._wgrad_ws = self._wgrad_wss[0]
        self._heads_ws = torch.empty(self.hip.heads_wgrad_workspace_floats(self.A), dtype=torch.float32,
                                     device=self.device)
        self._fc1_ws = torch.empty(self.hip.fc1_bwd_workspace_floats(), dtype=torch.float32, device=self.device)
        self.repack()

    # ------------------------------------------------------------------ forward
    @staticmethod
    def _src(x: torch.Tensor, ids, idx, B: int):
        """(ptr, ids_ptr, idx_ptr) of a conv1 input: a dense u8 [B,4,84,84] stack, or the
        HBM frame ring ``x`` addressed by frame ids ``ids`` [*,4] (rows picked by ``idx``)."""
        assert x.dtype == torch.uint8 and x.is_contiguous()
        if ids is None:
            assert tuple(x.shape) == (B, 4, 84, 84)
            return x.data_ptr(), 0, 0
        assert ids.dtype == torch.int32 and ids.shape[-1] == 4 and x.shape[-1] == 84 * 84
        if idx is None:
            assert ids.shape[0] == B
        return x.data_ptr(), ids.data_ptr(), 0 if idx is None else idx.data_ptr()

    def _heads_tuple(self, ws: NetWorkspace) -> tuple:
        m = self.model
        return (ws.z.data_ptr(), m.advantage[0].bias.data_ptr(), m.value[0].bias.data_ptr(),
                m.advantage[2].weight.data_ptr(), m.advantage[2].bias.data_ptr(), m.value[2].weight.data_ptr(),
                m.value[2].bias.data_ptr(), ws.h.data_ptr() if ws.h is not None else 0, ws.q.data_ptr())

    def forward(self, x: torch.Tensor, ws: NetWorkspace, ids: torch.Tensor | None = None,
                idx: torch.Tensor | None = None, act: tuple | None = None) -> torch.Tensor:
        """Q for ``x`` into ``ws.q``; ``act`` = ``ActorShard.act_args()``: the heads kernel
        also writes the eps-greedy actions."""
        forward_multi([(self, x, ws, ids, idx)], act=act)
        return ws.q

    __call__ = forward

    # ------------------------------------------------------------------ backward
    def backward(self, dq: torch.Tensor, x: torch.Tensor, ws: NetWorkspace, ids: torch.Tensor | None = None,
                 idx: torch.Tensor | None = None) -> None:
        """Write dL/dparam for the pass held in ``ws`` (input ``x``/``ids``/``idx`` as in
        :meth:`forward`) into the model's ``.grad`` views, given dL/dQ ``dq``."""
        B, A = ws.B, self.A
        h, s, m = self.hip, self._s(), self.model
        if self._wgrad_ws is None:
            self.enable_backward()
        h.heads_bwd(dq.data_ptr(), ws.h.data_ptr(), m.advantage[2].weight.data_ptr(), m.value[2].weight.data_ptr(),
                    ws.dA.data_ptr(), ws.dz.data_ptr(), ws.dz_bf.data_ptr(), B, A, s)
        h.heads_wgrad(ws.dA.data_ptr(), ws.h.data_ptr(), ws.dz.data_ptr(), B, A, self._heads_ws.data_ptr(),
                      m.advantage[2].weight.grad.data_ptr(), m.advantage[2].bias.grad.data_ptr(),
                      m.value[2].weight.grad.data_ptr(), m.value[2].bias.grad.data_ptr(),
                      m.advantage[0].bias.grad.data_ptr(), m.value[0].bias.grad.data_ptr(), s)
        self.trunk_backward(x, ws, ids, idx)

    def heads_finalize_job(self, part: torch.Tensor, G: int):
        """grad_finalize job reducing ``G`` head/FC1-bias partial slabs (dqn_heads_bwd) into
        the model's head gradients."""
        m = self.model
        return self.hip.heads_finalize_job(G, self.A, part.data_ptr(), m.advantage[2].weight.grad.data_ptr(),
                                           m.advantage[2].bias.grad.data_ptr(), m.value[2].weight.grad.data_ptr(),
                                           m.value[2].bias.grad.data_ptr(), m.advantage[0].bias.grad.data_ptr(),
                                           m.value[0].bias.grad.data_ptr())

    def trunk_backward(self, x: torch.Tensor, ws: NetWorkspace, ids: torch.Tensor | None = None,
                       idx: torch.Tensor | None = None, extra_jobs=(), sumsq: torch.Tensor | None = None,
                       after_first=None) -> int:
        """FC1 + conv backward from ``ws.dz_bf`` (dL/dz, bf16); the weight-gradient partials
        of all layers (+ ``extra_jobs``) are reduced by ONE grad_finalize, which also writes
        per-workgroup sum-of-squares partials into ``sumsq`` (fp64) when given; returns
        their count.  ``after_first()`` runs right after the first launch (the FC1 backward):
        a forked branch captured there keeps the backward chain the graph's first child."""
        self._fc1_bwd(ws)
        if after_first is not None:
            after_first()
        jobs = self._conv_chain(x, ws, ids, idx) + self._fc_jobs()
        return self.hip.grad_finalize(jobs + list(extra_jobs), self._s(), 0 if sumsq is None else sumsq.data_ptr())

    def fc_backward(self, ws: NetWorkspace, extra_jobs=()) -> None:
        """Data-parallel split, part 1: FC1 backward and the finalize of the FC1 (+ head,
        via ``extra_jobs``) gradients -- everything past conv3 in the flat buffer, ~91% of
        its bytes -- so their all-reduce can start while :meth:`conv_backward` runs."""
        self._fc1_bwd(ws)
        self.hip.grad_finalize(self._fc_jobs() + list(extra_jobs), self._s(), 0)

    def conv_backward(self, x: torch.Tensor, ws: NetWorkspace, ids: torch.Tensor | None = None,
                      idx: torch.Tensor | None = None, after_first=None) -> None:
        """Data-parallel split, part 2: conv3..conv1 backward + their finalize (needs
        ``ws.dy3`` from :meth:`fc_backward`); ``after_first`` as in :meth:`trunk_backward`."""
        self.hip.grad_finalize(self._conv_chain(x, ws, ids, idx, after_first), self._s(), 0)

    def _fc1_bwd(self, ws: NetWorkspace) -> None:
        # FC1: dy3 = relu_mask(dz . W) and dW slabs in one launch
        if self._wgrad_ws is None:
            self.enable_backward()
        self.hip.fc1_bwd(ws.dz_bf.data_ptr(), ws.a3.data_ptr(), self.wfc1t.data_ptr(), ws.dy3.data_ptr(),
                         self._fc1_ws.data_ptr(), ws.B, self._s())

    def _fc_jobs(self) -> list:
        m = self.model
        return [self.hip.fc1_finalize_job(0, self._fc1_ws.data_ptr(), m.advantage[0].weight.grad.data_ptr()),
                self.hip.fc1_finalize_job(1, self._fc1_ws.data_ptr(), m.value[0].weight.grad.data_ptr())]

    def _conv_chain(self, x, ws: NetWorkspace, ids, idx, after_first=None) -> list:
        """conv3 .. conv1 MFMA wgrad (partials only) / dgrad, where dgrad applies the ReLU
        backward of the layer below in its coalesced epilogue (ws.dy2 / ws.dy1 are the
        masked gradients); returns the finalize jobs of the three layers."""
        B = ws.B
        xp, ip, jp = self._src(x, ids, idx, B)
        h, s, f = self.hip, self._s(), self.model.features
        w1, w2, w3 = (t.data_ptr() for t in self._wgrad_wss)
        h.conv_wgrad(3, ws.a2.data_ptr(), 0, 0, ws.dy3.data_ptr(), 0, B, w3, 0, 0, s)
        if after_first is not None:
            after_first()
        h.conv_dgrad(3, ws.dy3.data_ptr(), 0, self.w3t.data_ptr(), ws.dy2.data_ptr(), ws.a2.data_ptr(), B, s)
        h.conv_wgrad(2, ws.a1.data_ptr(), 0, 0, ws.dy2.data_ptr(), 0, B, w2, 0, 0, s)
        h.conv_dgrad(2, ws.dy2.data_ptr(), 0, self.w2t.data_ptr(), ws.dy1.data_ptr(), ws.a1.data_ptr(), B, s)
        h.conv_wgrad(1, xp, ip, jp, ws.dy1.data_ptr(), 0, B, w1, 0, 0, s)
        return [h.conv_finalize_job(k, B, wsp, f[2 * k - 2].weight.grad.data_ptr(), f[2 * k - 2].bias.grad.data_ptr())
                for k, wsp in ((3, w3), (2, w2), (1, w1))]


def forward_multi(passes, act: tuple | None = None, draw=None) -> None:
    """Run up to 3 forward passes ``(net, x, ws, ids, idx)`` (same batch size and action
    count; the nets may differ, e.g. online and target) with ONE launch per layer: conv1,
    conv2, conv3, FC1, heads = 5 kernels instead of 5 per pass.  Each kernel boundary
    costs ~4.5 us on MI355X (rocprofv3 trace), so the learner's three passes save ~45 us
    per step; the larger grids also amortise the per-workgroup weight staging."""
    passes = list(passes)
    if getattr(passes[0][0], "fp32", False):
        from .fused_f32 import forward_multi_f32
        return forward_multi_f32(passes, act=act, draw=draw)
    assert draw is None, "the PER draw folds into the fp32 conv1 launch only"
    assert 1 <= len(passes) <= 3
    net0 = passes[0][0]
    B, A = passes[0][2].B, net0.A
    h, s = net0.hip, net0._s()
    c1, c2, c3, fc, hd = [], [], [], [], []
    for net, x, ws, ids, idx in passes:
        assert ws.B == B and net.A == A, "one launch per layer needs a common batch and action count"
        xp, ip, jp = net._src(x, ids, idx, B)
        c1.append((xp, ip, jp, net.w1p.data_ptr(), net.b1.data_ptr(), ws.a1.data_ptr()))
        c2.append((ws.a1.data_ptr(), 0, 0, net.w2p.data_ptr(), net.b2.data_ptr(), ws.a2.data_ptr()))
        c3.append((ws.a2.data_ptr(), 0, 0, net.w3p.data_ptr(), net.b3.data_ptr(), ws.a3.data_ptr()))
        fc.append((ws.a3.data_ptr(), net.wfc1p.data_ptr(), ws.z.data_ptr()))
        hd.append(net._heads_tuple(ws))
    h.conv_fwd_multi(1, c1, B, s)
    h.conv_fwd_multi(2, c2, B, s)
    h.conv_fwd_multi(3, c3, B, s)
    nsplit = h.fc1_fwd_multi(fc, B, s)
    h.heads_fwd_multi(hd, nsplit, B, A, s, act)


DTYPES = ("fp32", "bf16")


def make_hip_net(model: DuelingDQN, dtype: str = "fp32"):
    """The HIP network for ``dtype``: "fp32" (reference precision, fp32 MFMA, the default)
    or "bf16" (bf16 MFMA operands, fp32 accumulation; opt-in fast mode)."""
    if dtype == "fp32":
        from .fused_f32 import F32DuelingNet
        return F32DuelingNet(model)
    if dtype == "bf16":
        return HipDuelingNet(model)
    raise ValueError(f"dtype must be one of {DTYPES}, got {dtype!r}")


def make_workspace(B: int, A: int, device, dtype: str = "fp32", keep_for_backward: bool = False):
    if dtype == "fp32":
        from .fused_f32 import F32Workspace
        return F32Workspace(B, A, device, keep_for_backward)
    if dtype == "bf16":
        return NetWorkspace(B, A, device, keep_for_backward)
    raise ValueError(f"dtype must be one of {DTYPES}, got {dtype!r}")
