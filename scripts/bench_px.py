#!/usr/bin/env python
"""Per-launch timing of the pre-split exact (px) forward GEMMs against the fp32-MFMA bodies at
the learner's shapes (3 problems x B).  ``python scripts/bench_px.py [--B 512] [--iters 50]
[--graph 1] [--terms 6,8]``; ``--graph 0`` launches eagerly (rocprofv3 --pmc)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from apex_amd import ops  # noqa: E402
from apex_amd.models.dqn import DuelingDQN  # noqa: E402
from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace, forward_multi_f32  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--B", type=int, default=512)
ap.add_argument("--graph", type=int, default=1)
ap.add_argument("--terms", default="0,6,8", help="0 = fp32 MFMA body, 6 / 8 = px term products")
ap.add_argument("--only", default=None)
ap.add_argument("--pipes", default="1", help="px pipeline forms to sweep (knob 21)")
ap.add_argument("--bwd", type=int, default=1, help="also time the backward (pxb with px on)")
a = ap.parse_args()
dev = torch.device("cuda")
hip = ops.hip()
B, A = a.B, 18
m = DuelingDQN.from_shapes((4, 84, 84), A).to(dev)
m.flatten_parameters()
F = 4 * B
frames = torch.randint(0, 256, (F, 84 * 84), dtype=torch.uint8, device=dev)
ids = torch.randint(0, F, (B, 4), dtype=torch.int32, device=dev)
idx = torch.randperm(B, device=dev).int()
f = m.features


def S() -> int:
    return torch.cuda.current_stream().cuda_stream


def time_fn(fn) -> float:
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if a.graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(a.iters):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0.record()
        g.replay()
        e1.record()
    else:
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
    torch.cuda.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / a.iters


P = 3 * B
FLOP = {1: 2 * P * 400 * 32 * 256, 2: 2 * P * 81 * 64 * 512, 3: 2 * P * 49 * 64 * 576, 4: 2 * P * 256 * 3136}
NAME = {1: "conv1_fwd", 2: "conv2_fwd", 3: "conv3_fwd", 4: "fc1_fwd"}
outs = {}
combos = [(t, p) for t in map(int, a.terms.split(",")) for p in (map(int, a.pipes.split(",")) if t else [0])]
for terms, pipe in combos:
    hip.f32_set_variant(19, {0: 0, 6: 1, 8: 2}[terms])
    hip.f32_set_variant(21, pipe)
    net = F32DuelingNet(m)
    wss = [F32Workspace(B, A, dev, keep_for_backward=(i == 0)) for i in range(3)]
    forward_multi_f32([(net, frames, w, ids, idx) for w in wss])
    torch.cuda.synchronize()
    px = terms > 0

    def set3(layer):
        out = []
        for ws in wss:
            if layer == 1:
                t = (frames.data_ptr(), ids.data_ptr(), idx.data_ptr(), f[0].weight.data_ptr(), 0, f[0].bias.data_ptr(),
                     ws.a1.data_ptr())
                t += (0, 0, ws.a1x.data_ptr(), 0, 0, ws.a1x.shape[1]) if px else ()
            elif layer == 2:
                t = (ws.a1.data_ptr(), 0, 0, net.w2p.data_ptr(), 0, f[2].bias.data_ptr(), ws.a2.data_ptr())
                t += (ws.a1x.data_ptr(), net.wx("w2p"), ws.a2x.data_ptr(), ws.a1x.shape[1], net.x_plane,
                      ws.a2x.shape[1]) if px else ()
            elif layer == 3:
                t = (ws.a2.data_ptr(), 0, 0, net.w3p.data_ptr(), 0, f[4].bias.data_ptr(), ws.a3.data_ptr())
                t += (ws.a2x.data_ptr(), net.wx("w3p"), ws.a3x.data_ptr(), ws.a2x.shape[1], net.x_plane,
                      ws.a3x.shape[1]) if px else ()
            else:
                t = (ws.a3.data_ptr(), 0, 0, net.wfc1p.data_ptr(), 0, 0, ws.z.data_ptr())
                t += (ws.a3x.data_ptr(), net.wx("wfc1p"), 0, ws.a3x.shape[1], net.x_plane, 0) if px else ()
            out.append(t)
        return out

    for layer in (1, 2, 3, 4):
        if a.only and a.only not in NAME[layer]:
            continue
        sets = set3(layer)
        fn = ((lambda s=sets, L=layer: hip.f32_conv_fwd_multi(L, s, B, S())) if layer < 4
              else (lambda s=sets: hip.f32_fc1_fwd_multi(s, B, S())))
        us = time_fn(fn)
        tf = FLOP[layer] / us / 1e6
        print(f"terms={terms} pipe={pipe} {NAME[layer]:10s} {us:8.2f} us  {tf:6.1f} fp32-equivalent TFLOP/s")
    outs[(terms, pipe)] = wss[0].z.clone()
    if a.bwd:  # backward: FC1 (dgrad + wgrad) and the conv chain (conv3 / conv2 pairs + conv1 wgrad)
        hip.f32_set_variant(20, 1 if px else 0)
        for p in m.parameters():
            p.grad = torch.zeros_like(p)
        netb = F32DuelingNet(m)
        netb.enable_backward(B)
        wb = F32Workspace(B, A, dev, keep_for_backward=True)
        forward_multi_f32([(netb, frames, wb, ids, idx)])
        wb.dz.normal_()
        wb.dz.mul_((wb.h > 0).float())
        if wb.pxb:
            hip.f32_split_planes(wb.dz.data_ptr(), wb.dzx.data_ptr(), B * 256, wb.dzx.shape[1], S())
        for nm, fn, flop in (("fc1_bwd", lambda: netb._fc1_bwd(wb), 2 * 2 * B * 256 * 3136),
                             ("conv_bwd", lambda: netb._conv_chain(frames, wb, ids, idx),
                              2 * 2 * B * (49 * 64 * 576 + 81 * 64 * 512) + 2 * B * 400 * 32 * 256)):
            us = time_fn(fn)
            print(f"terms={terms} pipe={pipe} pxb={int(wb.pxb)} {nm:10s} {us:8.2f} us  {flop / us / 1e6:6.1f} fp32-equivalent TFLOP/s")
        hip.f32_set_variant(20, 0)
hip.f32_set_variant(19, 0)
base = outs.get((0, 0))
for (t, p), z in outs.items():
    if base is not None and t:
        print(f"terms={t} pipe={p}: max |z - z_fp32| / max|z| = {float((z - base).abs().max() / base.abs().max()):.3e}")
