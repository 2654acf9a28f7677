#!/usr/bin/env python
"""Per-launch timing of the fp32 (reference-precision) network kernels at the learner's
shapes: forward launches with 3 problems x B (Q(s), Q(s'), Q_target(s')), backward at B.
TFLOP/s are fp32-equivalent (the GEMMs run on the bf16 matrix cores through the exact
three-term split; the percentage is of the 157.3 TF fp32 MFMA peak, for comparison).

``python scripts/bench_f32.py [--B 512] [--iters 50] [--only NAME] [--graph 1]`` prints
us/launch and achieved TFLOP/s (157.3 TF = fp32 MFMA peak); ``--graph 0`` launches
eagerly (for rocprofv3 --pmc, one dispatch per launch)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from apex_amd import ops  # noqa: E402
from apex_amd.models.dqn import DuelingDQN  # noqa: E402
from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--only", default=None)
ap.add_argument("--B", type=int, default=512)
ap.add_argument("--graph", type=int, default=1)
ap.add_argument("--json", action="store_true")
ap.add_argument("--rounds", type=int, default=1, help="time every case this many times, round-robin; report the median")
ap.add_argument("--c1-wgrad-s1", action="store_true", help="+ conv1 weight gradient at one sample per workgroup")
ap.add_argument("--tile1", action="store_true", help="+ the alternative tiles: conv2 forward 64x64, "
                                                   "conv2/conv3 input gradient BK 32")
ap.add_argument("--tile2", action="store_true", help="+ forward tiles: conv2 128x64 as 4x1 waves (32x64 each), "
                                                   "conv3 128x64 (2x2 waves) and 128x32 (4x1)")
ap.add_argument("--c1-grids", default="", help="extra conv1 forward cases at these workgroup counts")
ap.add_argument("--wgrad-targets", default="", help="extra conv2/conv3 backward cases at these wgrad workgroup "
                                                    "targets, e.g. 512,1024 (default plan: the plain cases)")
a = ap.parse_args()
dev = torch.device("cuda")
hip = ops.hip()
B, A = a.B, 18
m = DuelingDQN.from_shapes((4, 84, 84), A).to(dev)
m.flatten_parameters()
for p in m.parameters():
    p.grad = torch.zeros_like(p)
net = F32DuelingNet(m)
net.enable_backward(B)
F = 4 * B
frames = torch.randint(0, 256, (F, 84 * 84), dtype=torch.uint8, device=dev)
ids = torch.randint(0, F, (B, 4), dtype=torch.int32, device=dev)
idx = torch.randperm(B, device=dev).int()
wss = [F32Workspace(B, A, dev, keep_for_backward=(i == 0)) for i in range(3)]
f = m.features


def S() -> int:  # the CURRENT stream at launch time (graph capture runs on a side stream)
    return torch.cuda.current_stream().cuda_stream


def set3(layer):
    out = []
    for ws in wss:
        if layer == 1:
            out.append((frames.data_ptr(), ids.data_ptr(), idx.data_ptr(), f[0].weight.data_ptr(), 0,
                        f[0].bias.data_ptr(), ws.a1.data_ptr()))
        elif layer == 2:
            out.append((ws.a1.data_ptr(), 0, 0, net.w2p.data_ptr(), 0, f[2].bias.data_ptr(), ws.a2.data_ptr()))
        elif layer == 3:
            out.append((ws.a2.data_ptr(), 0, 0, net.w3p.data_ptr(), 0, f[4].bias.data_ptr(), ws.a3.data_ptr()))
        else:
            out.append((ws.a3.data_ptr(), 0, 0, net.wfc1p.data_ptr(), 0, 0, ws.z.data_ptr()))
    return out


from apex_amd.models.fused import forward_multi  # noqa: E402

forward_multi([(net, frames, wss[0], ids, idx), (net, frames, wss[1], ids, idx), (net, frames, wss[2], ids, idx)])
ws = wss[0]
ws.dz.normal_()
ws.dz.mul_((ws.h > 0).float())
w1, w2, w3 = net._wgrad_wss
P = 3 * B
cases = {
    "conv1_fwd": (lambda: hip.f32_conv_fwd_multi(1, set3(1), B, S()), 2 * P * 400 * 32 * 256),
    "conv2_fwd": (lambda: hip.f32_conv_fwd_multi(2, set3(2), B, S()), 2 * P * 81 * 64 * 512),
    "conv3_fwd": (lambda: hip.f32_conv_fwd_multi(3, set3(3), B, S()), 2 * P * 49 * 64 * 576),
    "fc1_fwd": (lambda: hip.f32_fc1_fwd_multi(set3(4), B, S()), 2 * P * 256 * 3136),
    "fc1_bwd": (lambda: hip.f32_fc1_bwd_split(ws.dz.data_ptr(), ws.a3.data_ptr(), net.wfc1p.data_ptr(),
                                              ws.dy3.data_ptr(), net._fc1_ws.data_ptr(), B, S()),
                2 * 2 * B * 256 * 3136),
    "conv3_bwd": (lambda: hip.f32_conv_bwd(3, ws.a2.data_ptr(), 0, 0, ws.dy3.data_ptr(), net.w3t.data_ptr(),
                                           ws.a2.data_ptr(), ws.dy2.data_ptr(), w3.data_ptr(), B, S()),
                  2 * 2 * B * 49 * 64 * 576),
    "conv2_bwd": (lambda: hip.f32_conv_bwd(2, ws.a1.data_ptr(), 0, 0, ws.dy2.data_ptr(), net.w2t.data_ptr(),
                                           ws.a1.data_ptr(), ws.dy1.data_ptr(), w2.data_ptr(), B, S()),
                  2 * 2 * B * 81 * 64 * 512),
    "finalize": (lambda: hip.grad_finalize(
        [hip.f32_conv_finalize_job(k, B, wsp.data_ptr(), f[2 * k - 2].weight.grad.data_ptr(),
                                   f[2 * k - 2].bias.grad.data_ptr()) for k, wsp in ((3, w3), (2, w2), (1, w1))],
        S(), 0), 1),
    "conv1_wgrad": (lambda: hip.f32_conv_bwd(1, frames.data_ptr(), ids.data_ptr(), idx.data_ptr(), ws.dy1.data_ptr(),
                                             0, 0, 0, w1.data_ptr(), B, S()), 2 * B * 400 * 32 * 256),
}
mismatch = set()
mismatch_check = []  # (reference case, variant case, output getter): outputs compared bit for bit
for tg in [int(x) for x in a.wgrad_targets.split(",") if x]:
    for L, xin, dyin, wt, dx in ((3, "a2", "dy3", net.w3t, "dy2"), (2, "a1", "dy2", net.w2t, "dy1")):
        wsx = torch.empty(hip.f32_wgrad_workspace_floats(L, B, tg), dtype=torch.float32, device=dev)
        flop = 2 * 2 * B * (49 * 64 * 576 if L == 3 else 81 * 64 * 512)
        cases[f"conv{L}_bwd@{tg}"] = (
            (lambda L=L, xin=xin, dyin=dyin, wt=wt, dx=dx, wsx=wsx, tg=tg: hip.f32_conv_bwd(
                L, getattr(ws, xin).data_ptr(), 0, 0, getattr(ws, dyin).data_ptr(), wt.data_ptr(),
                getattr(ws, xin).data_ptr(), getattr(ws, dx).data_ptr(), wsx.data_ptr(), B, S(), target=tg)), flop)
if a.c1_wgrad_s1:  # conv1 weight gradient, one sample per workgroup (+ its finalize)
    w1s = torch.empty(hip.f32_wgrad_workspace_floats(1, B, 1), dtype=torch.float32, device=dev)
    cases["conv1_wgrad@s1"] = ((lambda: hip.f32_conv_bwd(1, frames.data_ptr(), ids.data_ptr(), idx.data_ptr(),
                                                         ws.dy1.data_ptr(), 0, 0, 0, w1s.data_ptr(), B, S(), target=1)),
                               2 * B * 400 * 32 * 256)
    cases["finalize1@s1"] = ((lambda: hip.grad_finalize([hip.f32_conv_finalize_job(
        1, B, w1s.data_ptr(), f[0].weight.grad.data_ptr(), f[0].bias.grad.data_ptr(), target=1)], S(), 0)), 1)
    cases["finalize1"] = ((lambda: hip.grad_finalize([hip.f32_conv_finalize_job(
        1, B, w1.data_ptr(), f[0].weight.grad.data_ptr(), f[0].bias.grad.data_ptr())], S(), 0)), 1)
if a.tile1:
    cases["conv2_fwd@t1"] = ((lambda: hip.f32_conv_fwd_multi(2, set3(2), B, S(), tile=1)), 2 * P * 81 * 64 * 512)
    cases["conv3_bwd@t1"] = ((lambda: hip.f32_conv_bwd(3, ws.a2.data_ptr(), 0, 0, ws.dy3.data_ptr(), net.w3t.data_ptr(),
                                                       ws.a2.data_ptr(), ws.dy2.data_ptr(), w3.data_ptr(), B, S(),
                                                       tile=1)), 2 * 2 * B * 49 * 64 * 576)
    cases["conv2_bwd@t1"] = ((lambda: hip.f32_conv_bwd(2, ws.a1.data_ptr(), 0, 0, ws.dy2.data_ptr(), net.w2t.data_ptr(),
                                                       ws.a1.data_ptr(), ws.dy1.data_ptr(), w2.data_ptr(), B, S(),
                                                       tile=1)), 2 * 2 * B * 81 * 64 * 512)
if a.tile2:
    cases["conv2_fwd@t2"] = ((lambda: hip.f32_conv_fwd_multi(2, set3(2), B, S(), tile=2)), 2 * P * 81 * 64 * 512)
    cases["conv3_fwd@t2"] = ((lambda: hip.f32_conv_fwd_multi(3, set3(3), B, S(), tile=2)), 2 * P * 49 * 64 * 576)
    cases["conv3_fwd@t3"] = ((lambda: hip.f32_conv_fwd_multi(3, set3(3), B, S(), tile=3)), 2 * P * 49 * 64 * 576)
for cg in [int(x) for x in a.c1_grids.split(",") if x]:
    cases[f"conv1_fwd@g{cg}"] = ((lambda cg=cg: hip.f32_conv_fwd_multi(1, set3(1), B, S(), c1_grid=cg)),
                                 2 * P * 400 * 32 * 256)
for ref_name, var_name, get in mismatch_check:
    cases[ref_name][0]()
    torch.cuda.synchronize()
    ref_out = get().clone()
    cases[var_name][0]()
    torch.cuda.synchronize()
    if not torch.equal(ref_out, get()):
        mismatch.add(var_name)
        print(f"{var_name}: output differs from {ref_name}, max abs {(ref_out - get()).abs().max().item():.3g}")
res = {}
runs = [(name, fn, flop) for name, (fn, flop) in cases.items() if not a.only or a.only in name]
for _ in range(5):  # clocks up and caches warm before the first timed case (it read ~10 % slow)
    for name, fn, flop in runs:
        fn()
torch.cuda.synchronize()
graphs = {}
if a.graph:
    for name, fn, flop in runs:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(a.iters):
                fn()
        g.replay()
        graphs[name] = g
    torch.cuda.synchronize()
times = {name: [] for name, _, _ in runs}
for _ in range(a.rounds):  # round-robin: clock / thermal drift hits every case alike
    for name, fn, flop in runs:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if a.graph:
            e0.record()
            graphs[name].replay()
            e1.record()
        else:
            fn()
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
        torch.cuda.synchronize()
        times[name].append(1000.0 * e0.elapsed_time(e1) / a.iters)
for name, fn, flop in runs:
    ts = sorted(times[name])
    us = ts[len(ts) // 2]
    res[name] = {"us": round(us, 2), "tflops": round(flop / us / 1e6, 1), "pct_peak": round(flop / us / 1e6 / 1.573, 1)}
    if not a.json:
        mm = " MISMATCH" if name in mismatch else ""
        spread = f"  [{ts[0]:.1f}-{ts[-1]:.1f}]" if len(ts) > 1 else ""
        print(f"{name:12s}{mm} {us:8.2f} us  {flop / us / 1e6:6.1f} TFLOP/s  ({flop / us / 1e6 / 1.573:4.1f}% of 157.3)"
              f"{spread}")
if a.json:
    print(json.dumps(res))
tot = sum(r["us"] for r in res.values())
print(f"total {tot:.1f} us")
