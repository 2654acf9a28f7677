"""Reference-precision (fp32) HIP path of the dueling Q-network.

The reference computes every forward, backward and optimizer step in fp32
(origin_repo/learner.py:139-145, utils.py:64-97, model.py:31-68).  ``F32DuelingNet``
runs the same Nature-CNN dueling network on gfx950's exact-f32 matrix instructions
(``v_mfma_f32_32x32x2_f32``, a k-ordered fmaf chain) -- ``ops/csrc/f32_kernels.hip``:

  forward (per layer ONE launch for up to 3 passes: Q(s), Q(s'), Q_target(s'))
    conv1   u8 frames (frame ring by id, converted in the loader) -> a1 fp32 NHWC
    conv2/3 implicit-GEMM, bias+ReLU fused -> a2, a3 fp32 NHWC
    fc1     split-K (7 slabs) -> heads_fwd (fp32 heads + dueling combine, shared with bf16)
  backward (4 GEMM launches + one grad_finalize)
    fc1 dgrad (ReLU mask fused) + fc1 wgrad (reference layout, written in place)
    conv3 wgrad partials + conv3 dgrad      (one launch)
    conv2 wgrad partials + conv2 dgrad      (one launch, stride-2 sub-pixel classes)
    conv1 wgrad partials from the u8 frames
    grad_finalize: deterministic partial reduce -> reference layout + bias grads + grad-norm partials

Weights are read from EXACT fp32 copies in GEMM layouts (one fp32 arena, see ``LAYOUT``):
k-contiguous rows for the forward B operands, co-contiguous transposes for the conv input
gradients.  The fused optimizer rewrites them in the same pass as the fp32 master update
(``pack_maps`` -> PackMap.arena_f32, FC1 through the LDS-tiled FcPack path), target sync and
actor publish copy arenas (``copy_packed_from``), and ``repack()`` re-derives the arena from
the master (init, broadcast, checkpoint load).  The master parameters stay the reference
state_dict; the arena only changes memory order, never a value.
"""
from __future__ import annotations

import torch

from .. import ops
from .dqn import DuelingDQN

P3, C3 = 49, 64
FEAT = P3 * C3  # 3136
F32_SPLITS = 7  # FC1 forward split-K slabs (f32_kernels.hip kFcSplits)


class F32Workspace:
    """fp32 activation buffers for one forward pass of batch ``B`` (+ backward buffers)."""

    def __init__(self, B: int, A: int, device, keep_for_backward: bool = False):
        self.B, self.A = B, A
        f32 = dict(dtype=torch.float32, device=device)
        self.a1 = torch.empty(B, 400, 32, **f32)
        self.a2 = torch.empty(B, 81, 64, **f32)
        self.a3 = torch.empty(B, FEAT, **f32)
        self.z = torch.empty(F32_SPLITS, B, 256, **f32)
        self.h = torch.empty(B, 256, **f32) if keep_for_backward else None
        self.q = torch.empty(B, A, **f32)
        if keep_for_backward:
            self.dA = torch.empty(B, A + 1, **f32)
            self.dz = torch.empty(B, 256, **f32)
            self.dz_bf = torch.empty(B, 256, dtype=torch.bfloat16, device=device)  # heads_bwd writes both
            self.dy3 = torch.empty(B, FEAT, **f32)
            self.dy2 = torch.empty(B, 81, 64, **f32)
            self.dy1 = torch.empty(B, 400, 32, **f32)


class F32DuelingNet:
    """fp32 MFMA kernels over a :class:`DuelingDQN` (fp32 master params, reference layout)."""

    fp32 = True
    # fp32 arena: forward layouts first (all an actor / target net needs), then the transposes
    LAYOUT = (("w2p", (64, 4, 4, 32)), ("w3p", (64, 3, 3, 64)), ("wfc1p", (256, P3, C3)),
              ("w2t", (4, 4, 32, 64)), ("w3t", (3, 3, 64, 64)))

    def __init__(self, model: DuelingDQN):
        assert model.cnn and tuple(model.input_shape) == (4, 84, 84), "HIP path is the Atari Nature-CNN"
        self.hip = ops.hip()
        assert self.hip.f32_fc1_splits() == F32_SPLITS
        self.model = model
        self.A = model.num_actions
        self.device = next(model.parameters()).device
        self._ws_B = None
        self._heads_ws = None
        self._maps = None
        sizes = [int(torch.Size(sh).numel()) for _, sh in self.LAYOUT]
        self.arena = torch.empty(sum(sizes), dtype=torch.float32, device=self.device)
        self.arena_offsets = {}
        off = 0
        for (name, sh), n in zip(self.LAYOUT, sizes):
            setattr(self, name, self.arena[off:off + n].view(sh))
            self.arena_offsets[name] = off
            off += n
        self.fwd_numel = self.arena_offsets["w2t"]
        self.repack()

    def repack(self) -> None:
        """Re-derive every packed copy from the fp32 master (exact: a permutation)."""
        f, m = self.model.features, self.model
        with torch.no_grad():
            self.w2p.copy_(f[2].weight.permute(0, 2, 3, 1))
            self.w3p.copy_(f[4].weight.permute(0, 2, 3, 1))
            self.wfc1p[:128].copy_(m.advantage[0].weight.view(128, C3, P3).permute(0, 2, 1))
            self.wfc1p[128:].copy_(m.value[0].weight.view(128, C3, P3).permute(0, 2, 1))
            self.w2t.copy_(f[2].weight.permute(2, 3, 1, 0))
            self.w3t.copy_(f[4].weight.permute(2, 3, 1, 0))

    def copy_packed_from(self, other: "F32DuelingNet", forward_only: bool = True) -> None:
        """Device copy of another net's packed weights (same architecture)."""
        n = self.fwd_numel if forward_only else self.arena.numel()
        self.arena[:n].copy_(other.arena[:n])

    def pack_maps(self) -> tuple[torch.Tensor, torch.Tensor]:
        """int32 (dst1, dst2) over the flat parameter order: arena positions of the packed
        copies of each conv weight element (-1: none; FC1 goes through ``fc_pack_args``)."""
        if self._maps is not None:
            return self._maps
        seg = {name: (o, n) for name, o, n in self.model.param_segments()}
        P = sum(n for _, n in seg.values())
        dst1 = torch.full((P,), -1, dtype=torch.int64)
        dst2 = torch.full((P,), -1, dtype=torch.int64)
        ao = self.arena_offsets
        for pname, N, C, K, fwd, bwd in (("features.2.weight", 64, 32, 4, "w2p", "w2t"),
                                         ("features.4.weight", 64, 64, 3, "w3p", "w3t")):
            o, n = seg[pname]
            ref = torch.arange(N * C * K * K).view(N, C, K, K)  # reference position of each element
            # packed position q holds reference element ref_order[q]
            for dst, order, base in ((dst1, ref.permute(0, 2, 3, 1).reshape(-1), ao[fwd]),
                                     (dst2, ref.permute(2, 3, 1, 0).reshape(-1), ao[bwd])):
                dst[o + order] = base + torch.arange(n)
        self._maps = (dst1.to(torch.int32).to(self.device), dst2.to(torch.int32).to(self.device))
        return self._maps

    def fc_pack_args(self) -> dict:
        """Optimizer FC1 tile path (FcPack, fp32): flat offsets of both FC1 weights and wfc1p."""
        seg = {name: o for name, o, _ in self.model.param_segments()}
        return {"fc_off0": seg["advantage.0.weight"], "fc_off1": seg["value.0.weight"],
                "fc_wp_f32": self.wfc1p.data_ptr()}

    def opt_pack_args(self) -> dict:
        d1, d2 = self.pack_maps()
        return {"dst1": d1.data_ptr(), "dst2": d2.data_ptr(), "arena_f32": self.arena.data_ptr(),
                **self.fc_pack_args()}

    @staticmethod
    def _s() -> int:
        return torch.cuda.current_stream().cuda_stream

    def enable_backward(self, B: int = 512) -> None:
        """Allocate the wgrad partial workspaces for batch ``B`` (call before graph capture)."""
        if self._ws_B == B:
            return
        h = self.hip
        self._wgrad_wss = [torch.empty(h.f32_wgrad_workspace_floats(k, B), dtype=torch.float32, device=self.device)
                           for k in (1, 2, 3)]
        self._heads_ws = torch.empty(h.heads_wgrad_workspace_floats(self.A), dtype=torch.float32, device=self.device)
        # FC1 weight gradient: natural-order batch-slice partials, transposed by grad_finalize
        self._fc1_G = h.f32_fc1_wgrad_slices(B)
        self._fc1_ws = torch.empty(h.f32_fc1_wgrad_workspace_floats(), dtype=torch.float32, device=self.device)
        self._ws_B = B

    # ------------------------------------------------------------------ forward
    @staticmethod
    def _src(x: torch.Tensor, ids, idx, B: int):
        assert x.dtype == torch.uint8 and x.is_contiguous()
        if ids is None:
            assert tuple(x.shape) == (B, 4, 84, 84)
            return x.data_ptr(), 0, 0
        assert ids.dtype == torch.int32 and ids.shape[-1] == 4 and x.shape[-1] == 84 * 84
        if idx is None:
            assert ids.shape[0] == B
        return x.data_ptr(), ids.data_ptr(), 0 if idx is None else idx.data_ptr()

    def _heads_tuple(self, ws: F32Workspace) -> tuple:
        m = self.model
        return (ws.z.data_ptr(), m.advantage[0].bias.data_ptr(), m.value[0].bias.data_ptr(),
                m.advantage[2].weight.data_ptr(), m.advantage[2].bias.data_ptr(), m.value[2].weight.data_ptr(),
                m.value[2].bias.data_ptr(), ws.h.data_ptr() if ws.h is not None else 0, ws.q.data_ptr())

    def forward(self, x: torch.Tensor, ws: F32Workspace, ids: torch.Tensor | None = None,
                idx: torch.Tensor | None = None, act: tuple | None = None) -> torch.Tensor:
        forward_multi_f32([(self, x, ws, ids, idx)], act=act)
        return ws.q

    __call__ = forward

    # ------------------------------------------------------------------ backward
    def backward(self, dq: torch.Tensor, x: torch.Tensor, ws: F32Workspace, ids: torch.Tensor | None = None,
                 idx: torch.Tensor | None = None) -> None:
        """dL/dparam for the pass held in ``ws`` into the model's ``.grad`` views, given dL/dQ."""
        B, A = ws.B, self.A
        h, s, m = self.hip, self._s(), self.model
        self.enable_backward(B)
        h.heads_bwd(dq.data_ptr(), ws.h.data_ptr(), m.advantage[2].weight.data_ptr(), m.value[2].weight.data_ptr(),
                    ws.dA.data_ptr(), ws.dz.data_ptr(), ws.dz_bf.data_ptr(), B, A, s)
        h.heads_wgrad(ws.dA.data_ptr(), ws.h.data_ptr(), ws.dz.data_ptr(), B, A, self._heads_ws.data_ptr(),
                      m.advantage[2].weight.grad.data_ptr(), m.advantage[2].bias.grad.data_ptr(),
                      m.value[2].weight.grad.data_ptr(), m.value[2].bias.grad.data_ptr(),
                      m.advantage[0].bias.grad.data_ptr(), m.value[0].bias.grad.data_ptr(), s)
        self.trunk_backward(x, ws, ids, idx)

    def heads_finalize_job(self, part: torch.Tensor, G: int):
        m = self.model
        return self.hip.heads_finalize_job(G, self.A, part.data_ptr(), m.advantage[2].weight.grad.data_ptr(),
                                           m.advantage[2].bias.grad.data_ptr(), m.value[2].weight.grad.data_ptr(),
                                           m.value[2].bias.grad.data_ptr(), m.advantage[0].bias.grad.data_ptr(),
                                           m.value[0].bias.grad.data_ptr())

    fc1_ride_ok = True  # the backward launches take priority-tree riders (ops/csrc/tree_dev.h)

    def _fc1_bwd(self, ws: F32Workspace, ride=None) -> list:
        """FC1 dgrad + weight gradient (one launch, + the tree-write rider ``ride``); returns
        the finalize jobs that complete the weight gradient (sum the slices + transpose to the
        reference layout, with their sum-of-squares partials)."""
        m = self.model
        ga, gv = m.advantage[0].weight.grad, m.value[0].weight.grad
        self.hip.f32_fc1_bwd_split(ws.dz.data_ptr(), ws.a3.data_ptr(), self.wfc1p.data_ptr(), ws.dy3.data_ptr(),
                                   self._fc1_ws.data_ptr(), ws.B, self._s(), ride=ride)
        return [self.hip.f32_fc1_finalize_job(0, self._fc1_G, self._fc1_ws.data_ptr(), ga.data_ptr()),
                self.hip.f32_fc1_finalize_job(1, self._fc1_G, self._fc1_ws.data_ptr(), gv.data_ptr())]

    def _conv_chain(self, x, ws: F32Workspace, ids, idx, after_first=None, rides=(None, None)) -> list:
        """conv3 .. conv1 backward (wgrad partials + masked dgrad per launch; ``rides``: the
        tree-write riders of the conv3 / conv2 launches); returns the finalize jobs of the
        three layers."""
        B = ws.B
        h, s, f = self.hip, self._s(), self.model.features
        xp, ip, jp = self._src(x, ids, idx, B)
        w1, w2, w3 = self._wgrad_wss
        h.f32_conv_bwd(3, ws.a2.data_ptr(), 0, 0, ws.dy3.data_ptr(), self.w3t.data_ptr(), ws.a2.data_ptr(),
                       ws.dy2.data_ptr(), w3.data_ptr(), B, s, ride=rides[0])
        if after_first is not None:
            after_first()
        h.f32_conv_bwd(2, ws.a1.data_ptr(), 0, 0, ws.dy2.data_ptr(), self.w2t.data_ptr(), ws.a1.data_ptr(),
                       ws.dy1.data_ptr(), w2.data_ptr(), B, s, ride=rides[1])
        h.f32_conv_bwd(1, xp, ip, jp, ws.dy1.data_ptr(), 0, 0, 0, w1.data_ptr(), B, s)
        return [h.f32_conv_finalize_job(k, B, wsp.data_ptr(), f[2 * k - 2].weight.grad.data_ptr(),
                                        f[2 * k - 2].bias.grad.data_ptr()) for k, wsp in ((3, w3), (2, w2), (1, w1))]

    def fc_backward(self, ws: F32Workspace, extra_jobs=()) -> None:
        """Data-parallel split, part 1: the FC1 backward + the finalize of its slices and of
        ``extra_jobs`` (the heads), so the FC1/head all-reduce can start while
        :meth:`conv_backward` runs."""
        self.enable_backward(ws.B)
        self.hip.grad_finalize(self._fc1_bwd(ws) + list(extra_jobs), self._s(), 0)

    def conv_backward(self, x: torch.Tensor, ws: F32Workspace, ids: torch.Tensor | None = None,
                      idx: torch.Tensor | None = None, after_first=None) -> None:
        """Data-parallel split, part 2: conv3..conv1 backward + their finalize."""
        self.hip.grad_finalize(self._conv_chain(x, ws, ids, idx, after_first), self._s(), 0)

    def trunk_backward(self, x: torch.Tensor, ws: F32Workspace, ids: torch.Tensor | None = None,
                       idx: torch.Tensor | None = None, extra_jobs=(), sumsq: torch.Tensor | None = None,
                       after_first=None, rides=(None, None, None, None)) -> int:
        """FC1 + conv backward from ``ws.dz`` (fp32 dL/dz).  The conv weight-gradient
        partials (+ ``extra_jobs``) are reduced by ONE grad_finalize, which also writes the
        per-workgroup sum-of-squares partials of EVERY gradient into ``sumsq`` (fp64) when
        given; returns the partial count.  ``after_first()`` runs right after the first launch;
        ``rides`` = the priority-tree riders of the FC1, conv3 and conv2 launches and the finalize."""
        self.enable_backward(ws.B)
        fc1_jobs = self._fc1_bwd(ws, ride=rides[0])
        if after_first is not None:
            after_first()
        h = self.hip
        jobs = self._conv_chain(x, ws, ids, idx, rides=rides[1:3]) + list(extra_jobs) + fc1_jobs
        return h.grad_finalize(jobs, self._s(), 0 if sumsq is None else sumsq.data_ptr(), ride=rides[3])


def forward_multi_f32(passes, act: tuple | None = None, draw=None) -> None:
    """Up to 3 fp32 forward passes ``(net, x, ws, ids, idx)`` (common batch and action
    count; the nets may differ, e.g. online and target) with ONE launch per layer.  ``draw``
    (``make_conv_sample``): the conv1 launch draws the PER rows that ``idx`` then holds."""
    passes = list(passes)
    assert 1 <= len(passes) <= 3
    net0 = passes[0][0]
    B, A = passes[0][2].B, net0.A
    h, s = net0.hip, net0._s()
    c1, c2, c3, fc, hd = [], [], [], [], []
    for net, x, ws, ids, idx in passes:
        assert ws.B == B and net.A == A, "one launch per layer needs a common batch and action count"
        m, f = net.model, net.model.features
        xp, ip, jp = net._src(x, ids, idx, B)
        c1.append((xp, ip, jp, f[0].weight.data_ptr(), 0, f[0].bias.data_ptr(), ws.a1.data_ptr()))
        c2.append((ws.a1.data_ptr(), 0, 0, net.w2p.data_ptr(), 0, f[2].bias.data_ptr(), ws.a2.data_ptr()))
        c3.append((ws.a2.data_ptr(), 0, 0, net.w3p.data_ptr(), 0, f[4].bias.data_ptr(), ws.a3.data_ptr()))
        fc.append((ws.a3.data_ptr(), 0, 0, net.wfc1p.data_ptr(), 0, 0, ws.z.data_ptr()))
        hd.append(net._heads_tuple(ws))
    h.f32_conv_fwd_multi(1, c1, B, s, draw=draw)
    h.f32_conv_fwd_multi(2, c2, B, s)
    h.f32_conv_fwd_multi(3, c3, B, s)
    nsplit = h.f32_fc1_fwd_multi(fc, B, s)
    h.heads_fwd_multi(hd, nsplit, B, A, s, act)
