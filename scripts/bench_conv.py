"""Per-kernel timing of the MFMA conv / heads kernels at the learner batch (B=512).

``python scripts/bench_conv.py [--iters N] [--only NAME]`` prints us/call from HIP
events around N back-to-back launches (no graph), for use with rocprofv3 --pmc.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from apex_amd import ops  # noqa: E402
from apex_amd.models.dqn import DuelingDQN  # noqa: E402
from apex_amd.models.fused import HipDuelingNet, NetWorkspace  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=100)
ap.add_argument("--only", default=None)
ap.add_argument("--B", type=int, default=512)
ap.add_argument("--graph", type=int, default=1, help="time a captured graph of --iters launches (no launch overhead)")
a = ap.parse_args()
dev = torch.device("cuda")
hip = ops.hip()
B = a.B
m = DuelingDQN.from_shapes((4, 84, 84), 18).to(dev)
m.flatten_parameters()
for p in m.parameters():
    p.grad = torch.zeros_like(p)
net = HipDuelingNet(m)
net.enable_backward()
ws = NetWorkspace(B, 18, dev, keep_for_backward=True)
x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=dev)
F = 3 * B
frames = torch.randint(0, 256, (F, 84 * 84), dtype=torch.uint8, device=dev)
ids = torch.randint(0, F, (B, 4), dtype=torch.int32, device=dev)
idx = torch.randperm(B, device=dev).int()
s = torch.cuda.current_stream().cuda_stream
f = m.features
net(x, ws)
dq = torch.randn(B, 18, device=dev)
net.backward(dq, x, ws)
wsp = net._wgrad_wss[2].data_ptr()
fin_jobs = [hip.conv_finalize_job(k, B, net._wgrad_wss[k - 1].data_ptr(), m.features[2 * k - 2].weight.grad.data_ptr(),
                                  m.features[2 * k - 2].bias.grad.data_ptr()) for k in (3, 2, 1)]
fin_jobs += [hip.fc1_finalize_job(0, net._fc1_ws.data_ptr(), m.advantage[0].weight.grad.data_ptr()),
             hip.fc1_finalize_job(1, net._fc1_ws.data_ptr(), m.value[0].weight.grad.data_ptr())]

cases = {
    "conv1_fwd_dense": lambda: hip.conv_fwd(1, x.data_ptr(), 0, 0, net.w1p.data_ptr(), net.b1.data_ptr(),
                                            ws.a1.data_ptr(), B, s),
    "conv1_fwd_ring": lambda: hip.conv_fwd(1, frames.data_ptr(), ids.data_ptr(), idx.data_ptr(), net.w1p.data_ptr(),
                                           net.b1.data_ptr(), ws.a1.data_ptr(), B, s),
    "conv2_fwd": lambda: hip.conv_fwd(2, ws.a1.data_ptr(), 0, 0, net.w2p.data_ptr(), net.b2.data_ptr(),
                                      ws.a2.data_ptr(), B, s),
    "conv3_fwd": lambda: hip.conv_fwd(3, ws.a2.data_ptr(), 0, 0, net.w3p.data_ptr(), net.b3.data_ptr(),
                                      ws.a3.data_ptr(), B, s),
    "fc1_fwd": lambda: hip.fc1_fwd(ws.a3.data_ptr(), net.wfc1p.data_ptr(), ws.z.data_ptr(), B, s),
    "fc1_fwd_blaslt": lambda: torch.mm(ws.a3, net.wfc1p.t(), out_dtype=torch.float32, out=ws.z[0]),
    "heads_fwd": lambda: hip.heads_fwd(ws.z.data_ptr(), hip.fc1_splits_for(B), m.advantage[0].bias.data_ptr(), m.value[0].bias.data_ptr(),
                                       m.advantage[2].weight.data_ptr(), m.advantage[2].bias.data_ptr(),
                                       m.value[2].weight.data_ptr(), m.value[2].bias.data_ptr(), ws.h.data_ptr(),
                                       ws.q.data_ptr(), B, 18, s),
    "wgrad3": lambda: hip.conv_wgrad(3, ws.a2.data_ptr(), 0, 0, ws.dy3.data_ptr(), 0, B, wsp,
                                     f[4].weight.grad.data_ptr(), f[4].bias.grad.data_ptr(), s),
    "dgrad3": lambda: hip.conv_dgrad(3, ws.dy3.data_ptr(), 0, net.w3t.data_ptr(), ws.dy2.data_ptr(),
                                     ws.a2.data_ptr(), B, s),
    "wgrad2": lambda: hip.conv_wgrad(2, ws.a1.data_ptr(), 0, 0, ws.dy2.data_ptr(), 0, B, wsp,
                                     f[2].weight.grad.data_ptr(), f[2].bias.grad.data_ptr(), s),
    "dgrad2": lambda: hip.conv_dgrad(2, ws.dy2.data_ptr(), 0, net.w2t.data_ptr(), ws.dy1.data_ptr(),
                                     ws.a1.data_ptr(), B, s),
    "wgrad1": lambda: hip.conv_wgrad(1, x.data_ptr(), 0, 0, ws.dy1.data_ptr(), 0, B, wsp,
                                     f[0].weight.grad.data_ptr(), f[0].bias.grad.data_ptr(), s),
    "fc1_bwd": lambda: hip.fc1_bwd(ws.dz_bf.data_ptr(), ws.a3.data_ptr(), net.wfc1t.data_ptr(), ws.dy3.data_ptr(),
                                   net._fc1_ws.data_ptr(), B, s),
    "finalize_all": lambda: hip.grad_finalize(fin_jobs, s),
}
flat = m._flat if getattr(m, "_flat", None) is not None else m.flatten_parameters()
P = flat.numel()
gflat = torch.randn(P, device=dev) * 1e-3
s1o, s2o = torch.zeros(P, device=dev), torch.zeros(P, device=dev)
parts = torch.rand(1518, dtype=torch.float64, device=dev)
norms = torch.zeros(4, device=dev)
stp = torch.zeros(1, dtype=torch.int64, device=dev)
d1, d2 = net.pack_maps()
hp = hip.RMSpropParams(6.25e-5, 0.95, 1.5e-7, 40.0, 1.0, 0, 0, True)
fcargs = net.fc_pack_args()
cases["opt_rmsprop_tiles"] = lambda: hip.rmsprop_step(flat.data_ptr(), gflat.data_ptr(), s1o.data_ptr(), s2o.data_ptr(), P,
                                                      parts.data_ptr(), parts.numel(), hp, stp.data_ptr(),
                                                      norms.data_ptr(), s, d1.data_ptr(), d2.data_ptr(),
                                                      net.arena.data_ptr(), **fcargs)
cases["opt_rmsprop_scatter"] = lambda: hip.rmsprop_step(flat.data_ptr(), gflat.data_ptr(), s1o.data_ptr(),
                                                        s2o.data_ptr(), P, parts.data_ptr(), parts.numel(), hp,
                                                        stp.data_ptr(), norms.data_ptr(), s, d1.data_ptr(),
                                                        d2.data_ptr(), net.arena.data_ptr())
cases["opt_rmsprop_nopack"] = lambda: hip.rmsprop_step(flat.data_ptr(), gflat.data_ptr(), s1o.data_ptr(),
                                                       s2o.data_ptr(), P, parts.data_ptr(), parts.numel(), hp,
                                                       stp.data_ptr(), norms.data_ptr(), s)
cases["grad_sumsq"] = lambda: hip.grad_sumsq(gflat.data_ptr(), P, parts.data_ptr(), s)
flops = {"conv1": 2 * 3.28e6, "conv2": 2 * 2.65e6, "conv3": 2 * 1.81e6}
for name, fn in cases.items():
    if a.only and a.only not in name:
        continue
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    if a.graph:
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            s = torch.cuda.current_stream().cuda_stream
            with torch.cuda.graph(g, stream=cs):
                for _ in range(a.iters):
                    fn()
        torch.cuda.current_stream().wait_stream(cs)
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
    us = e0.elapsed_time(e1) / a.iters * 1000
    fl = flops.get(name[:5], 0) * B
    print(f"{name:18s} {us:8.2f} us" + (f"  {fl / us / 1e6:7.1f} TFLOP/s" if fl else ""), flush=True)
