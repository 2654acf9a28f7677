#!/usr/bin/env python
"""Per-tensor gradient accuracy of ONE fp32 HIP learner step vs fp64 PyTorch on the same batch
(and PyTorch fp32's own error for scale): which layer's gradient lost precision.

Prints, per parameter: ||g_hip - g64|| / ||g64||, ||g_t32 - g64|| / ||g64||, and the count of
elements whose sign differs from fp64 while |g64| > 1e-8 (RMSprop's first steps are sign-like).
``python scripts/diag/grad_check.py [--B 256]``"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    a = ap.parse_args()
    from apex_amd.algo.losses import compute_loss_device
    from apex_amd.engine.apex import ApexEngine, EngineConfig
    from apex_amd.engine.learner import LearnerConfig
    from apex_amd.models.dqn import DuelingDQN

    cuda = torch.device("cuda")
    lc = LearnerConfig(batch_size=a.B, forward="hip", dtype="fp32")
    cfg = EngineConfig(n_envs=64, replay_capacity=16384, threshold_size=8192, learner=lc)
    eng = ApexEngine(cfg, cuda)
    eng.fill()
    L, rp = eng.learner, eng.replay

    def clone(src, dt):
        m = DuelingDQN.from_shapes((4, 84, 84), cfg.n_actions).to(cuda)
        m.load_state_dict(src.state_dict())
        return m.to(dt)

    m64, t64 = clone(L.model, torch.float64), clone(L.target, torch.float64)
    m32, t32 = clone(L.model, torch.float32), clone(L.target, torch.float32)
    p_before = {n: p.detach().double().clone() for n, p in L.model.named_parameters()}
    L.step()
    torch.cuda.synchronize()
    B = a.B
    s = torch.empty(B, 4, 84, 84, dtype=torch.uint8, device=cuda)
    s2 = torch.empty_like(s)
    act = torch.empty(B, dtype=torch.int32, device=cuda)
    r = torch.empty(B, device=cuda)
    d = torch.empty(B, device=cuda)
    rp.gather(L.idx, s, s2, act, r, d)
    grads = {}
    for name, (m, t, dt) in (("t64", (m64, t64, torch.float64)), ("t32", (m32, t32, torch.float32))):
        batch = (s.to(dt), act.long(), r.to(dt), s2.to(dt), d.to(dt), L.w.to(dt))
        loss, _ = compute_loss_device(m, t, batch, lc.n_step, lc.gamma)
        m.zero_grad()
        loss.backward()
        grads[name] = {n: p.grad.detach().double() for n, p in m.named_parameters()}
    # forward activations of the s pass (ws_s: channels-last) vs fp64 / fp32 torch on the same states
    with torch.no_grad():
        acts = {}
        for name, m, dt in (("t64", m64, torch.float64), ("t32", m32, torch.float32)):
            x = s.to(dt) / 255.0 if getattr(m, "scale_input", False) else s.to(dt)
            f = m.features
            a1 = f[1](f[0](x)); a2 = f[3](f[2](a1)); a3 = f[5](f[4](a2))
            acts[name] = {"a1": a1.permute(0, 2, 3, 1).reshape(B, 400, 32).double(),
                          "a2": a2.permute(0, 2, 3, 1).reshape(B, 81, 64).double(),
                          "q": m(x).double()}
        ws = L.ws_s
        hip_acts = {"a1": ws.a1.double(), "a2": ws.a2.double(), "q": ws.q.double()}
        for k in ("a1", "a2", "q"):
            ref = acts["t64"][k]
            den = ref.norm().item() + 1e-30
            print(f"fwd {k}: hip rel {(hip_acts[k] - ref).norm().item() / den:.3g}  "
                  f"t32 rel {(acts['t32'][k] - ref).norm().item() / den:.3g}")
        # the s' passes and the TD error
        for name, m, t, dt in (("t64", m64, t64, torch.float64), ("t32", m32, t32, torch.float32)):
            acts[name]["q2"] = m(s2.to(dt)).double()
            acts[name]["q2t"] = t(s2.to(dt)).double()
        hip_acts["q2"], hip_acts["q2t"] = L.ws_s2.q.double(), L.ws_t.q.double()
        for k in ("q2", "q2t"):
            ref = acts["t64"][k]
            den = ref.norm().item() + 1e-30
            print(f"fwd {k}: hip rel {(hip_acts[k] - ref).norm().item() / den:.3g}  "
                  f"t32 rel {(acts['t32'][k] - ref).norm().item() / den:.3g}")
        ar = torch.arange(B, device=cuda)
        for name in ("t64", "t32"):
            q, q2, q2t = acts[name]["q"], acts[name]["q2"], acts[name]["q2t"]
            y = r.double() + (lc.gamma ** lc.n_step) * q2t[ar, q2.argmax(1)] * (1 - d.double())
            acts[name]["delta"] = (y - q[ar, act.long()]).abs()
        ref = acts["t64"]["delta"]
        print(f"delta: hip rel {(L.delta.double() - ref).norm().item() / ref.norm().item():.3g}  "
              f"t32 rel {(acts['t32']['delta'] - ref).norm().item() / ref.norm().item():.3g}  "
              f"hip max abs {(L.delta.double() - ref).abs().max().item():.3g}")
        print(f"gamma_n used {L.gamma_n!r} vs {lc.gamma ** lc.n_step!r}")
        am64 = acts["t64"]["q2"].argmax(1)
        print(f"argmax Q(s') differs from fp64: hip {int((hip_acts['q2'].argmax(1) != am64).sum())} "
              f"t32 {int((acts['t32']['q2'].argmax(1) != am64).sum())} of {B}")
        small = ref < 1.0  # the Huber-quadratic samples: their |td| IS the loss gradient
        yv, qa = {}, {}
        for name in ("t64", "t32", "hip"):
            src = acts[name] if name != "hip" else hip_acts
            q, q2, q2t = src["q"], src["q2"], src["q2t"]
            yv[name] = r.double() + (lc.gamma ** lc.n_step) * q2t[ar, q2.argmax(1)] * (1 - d.double())
            qa[name] = q[ar, act.long()]
        for name in ("hip", "t32"):
            dd = (yv[name] - qa[name]) - (yv["t64"] - qa["t64"])
            print(f"{name}: small-td samples {int(small.sum())}: |err td| rms {dd[small].pow(2).mean().sqrt().item():.3g} "
                  f"|err qa| rms {(qa[name] - qa['t64'])[small].pow(2).mean().sqrt().item():.3g} "
                  f"|err y| rms {(yv[name] - yv['t64'])[small].pow(2).mean().sqrt().item():.3g}")
        print(f"|Q| mean {qa['t64'].abs().mean().item():.4g}, |td| mean over small {ref[small].mean().item():.4g}")
        hd = (L.delta.double() - ref).abs()
        k = int(hd.argmax())
        print(f"worst delta sample {k}: hip {float(L.delta[k]):.7g} fp64 {float(ref[k]):.7g} "
              f"t32 {float(acts['t32']['delta'][k]):.7g}")
    st = L.stats()
    n64 = torch.sqrt(sum((g ** 2).sum() for g in grads["t64"].values())).item()
    print(f"grad norm: hip {st['grad_norm_l2']:.9g}  fp64 {n64:.9g}  (clip 40)")
    print(f"{'param':28s} {'hip rel':>10s} {'t32 rel':>10s} {'hip sign':>9s} {'t32 sign':>9s} {'|g64|':>10s}")
    for n, p in L.model.named_parameters():
        g = p.grad.detach().double()
        g64, g32 = grads["t64"][n], grads["t32"][n]
        den = g64.norm().item() + 1e-30
        big = g64.abs() > 1e-8
        sh = int(((torch.sign(g) != torch.sign(g64)) & big).sum())
        s3 = int(((torch.sign(g32) != torch.sign(g64)) & big).sum())
        print(f"{n:28s} {(g - g64).norm().item() / den:10.3g} {(g32 - g64).norm().item() / den:10.3g} "
              f"{sh:9d} {s3:9d} {den:10.3g}")
    # the first centered-RMSprop update from each gradient (clip inactive below 40), per tensor:
    # where do the HIP and fp64 updates differ, and how large are the gradients there
    lr, al, eps = lc.lr, lc.rms_alpha, lc.rms_eps
    print("update diff per tensor: ||dp_hip - dp_64|| / ||dp_64||, elements off by > 0.05 lr, their |g64| median")
    tot = 0.0
    for n, p in L.model.named_parameters():
        g64 = grads["t64"][n]
        sq, ga = (1 - al) * g64 * g64, (1 - al) * g64
        dp64 = -lr * g64 / (torch.sqrt(torch.clamp(sq - ga * ga, min=0)) + eps)
        dph = p.detach().double() - p_before[n]
        diff = (dph - dp64)
        off = diff.abs() > 0.05 * lr
        tot += float((diff ** 2).sum())
        med = float(g64[off].abs().median()) if off.any() else float("nan")
        print(f"{n:28s} {diff.norm().item() / (dp64.norm().item() + 1e-30):10.3g} {int(off.sum()):8d} {med:10.3g}")
    print(f"total update diff {tot ** 0.5:.4g}")


if __name__ == "__main__":
    main()
