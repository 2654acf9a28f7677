#!/usr/bin/env python
"""Time the fp32 DQN learner's step tail alone: grad_finalize (every job, and split into its
FC1 / conv+heads parts) and the centered-RMSprop launch (``DQNLearner.optimize``), each
replayed in a captured graph of 100 launches after real learner steps (timing only: the
optimizer state keeps moving, the numbers are launch durations)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402


def main():
    from apex_amd.engine.apex import ApexEngine, EngineConfig
    from apex_amd.engine.learner import LearnerConfig

    lc = LearnerConfig(batch_size=512, forward="hip", dtype="fp32")
    eng = ApexEngine(EngineConfig(learner=lc, threshold_size=8192), "cuda:0")
    eng.fill()
    for _ in range(3):
        eng.train_step()
    torch.cuda.synchronize()
    L = eng.learner
    net, h = L.net, L.hip
    B = L.cfg.batch_size
    f = net.model.features
    m = net.model
    w1, w2, w3 = net._wgrad_wss
    conv = [h.f32_conv_finalize_job(k, B, wsp.data_ptr(), f[2 * k - 2].weight.grad.data_ptr(),
                                    f[2 * k - 2].bias.grad.data_ptr()) for k, wsp in ((3, w3), (2, w2), (1, w1))]
    heads = [net.heads_finalize_job(L.lh_part, L.lh_blocks)]
    fc1 = [h.f32_fc1_finalize_job(0, net._fc1_G, net._fc1_ws.data_ptr(), m.advantage[0].weight.grad.data_ptr()),
           h.f32_fc1_finalize_job(1, net._fc1_G, net._fc1_ws.data_ptr(), m.value[0].weight.grad.data_ptr())]
    sq = L.fin_partials.data_ptr()
    for k in (1, 2, 3):
        print(f"conv{k} wgrad slices: {h.f32_wgrad_splits(k, B, 0)}")
    print(f"heads partial blocks: {L.lh_blocks}")
    S = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    cases = {
        "finalize (all jobs)": lambda: h.grad_finalize(conv + heads + fc1, S(), sq),
        "finalize (conv + heads)": lambda: h.grad_finalize(conv + heads, S(), sq),
        "finalize (FC1 only)": lambda: h.grad_finalize(fc1, S(), sq),
        "finalize (conv1 only)": lambda: h.grad_finalize(conv[2:], S(), sq),
        "finalize (conv2 only)": lambda: h.grad_finalize(conv[1:2], S(), sq),
        "finalize (conv3 only)": lambda: h.grad_finalize(conv[:1], S(), sq),
        "finalize (heads only)": lambda: h.grad_finalize(heads, S(), sq),
        "optimizer (RMSprop + packed copies)": L.optimize,
    }
    n = 100
    res = {}
    for rnd in range(3):
        for name, fn in cases.items():
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(n):
                    fn()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(name, []).append(1000 * e0.elapsed_time(e1) / n)
    for k, v in res.items():
        print(f"{k}: {sorted(v)[1]:.2f} us per launch  {['%.2f' % x for x in v]}")


if __name__ == "__main__":
    main()
