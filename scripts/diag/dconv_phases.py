#!/usr/bin/env python
"""Phase cycles of the sample-resident conv forward (f32_conv_fwd_direct_k, knob 25 = 4 | 5:
4 / 8 waves with s_memtime stamps): per wave, the cycles spent in the group-start DMA wait +
barrier, the DMA issue + deferred stores, the per-group setup, the MFMA step loop, and the
whole kernel -- mean over waves, at the learner's 3 x 512-sample launch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from apex_amd import ops  # noqa: E402
from apex_amd.models.dqn import DuelingDQN  # noqa: E402
from apex_amd.models.fused import forward_multi  # noqa: E402
from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace  # noqa: E402

dev = torch.device("cuda")
hip = ops.hip()
B = int(os.environ.get("B", "512"))
m = DuelingDQN.from_shapes((4, 84, 84), 18).to(dev)
m.flatten_parameters()
net = F32DuelingNet(m)
x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=dev)
wss = [F32Workspace(B, 18, dev) for _ in range(3)]
forward_multi([(net, x, w, None, None) for w in wss])
f = m.features
S = torch.cuda.current_stream().cuda_stream
names = ["wait+barrier", "dma issue+stores", "setup", "mfma steps", "total"]
for knob in (4, 5):
    hip.f32_set_variant(25, knob)
    for layer, a_in, wp, bias, a_out in ((2, "a1", net.w2p, f[2].bias, "a2"), (3, "a2", net.w3p, f[4].bias, "a3")):
        st = [torch.zeros(256 * 8 * 5, dtype=torch.int64, device=dev) for _ in range(3)]
        probs = [(getattr(w, a_in).data_ptr(), 0, 0, wp.data_ptr(), st[i].data_ptr(), bias.data_ptr(),
                  getattr(w, a_out).data_ptr()) for i, w in enumerate(wss)]
        for _ in range(200):  # hot clocks
            hip.f32_conv_fwd_multi(layer, probs, B, S)
        torch.cuda.synchronize()
        for s in st:
            s.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        hip.f32_conv_fwd_multi(layer, probs, B, S)
        e1.record()
        torch.cuda.synchronize()
        ph = torch.cat([s.view(-1, 5) for s in st]).double()
        ph = ph[ph[:, 4] > 0]
        mean = ph.mean(0).tolist()
        print(f"conv{layer} knob 25={knob}: {e0.elapsed_time(e1) * 1000:.1f} us, {len(ph)} waves; mean cycles: "
              + ", ".join(f"{n} {v:.0f} ({100 * v / mean[4]:.0f}%)" for n, v in zip(names, mean)))
hip.f32_set_variant(25, 0)
