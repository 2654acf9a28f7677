"""The HIP learner learns like the reference's fp32 PyTorch learner.

The reference learner step (origin_repo/learner.py:152-175, utils.py:64-97) is an fp32
``DuelingDQN`` + ``compute_loss`` + ``clip_grad_norm_(40)`` + centered ``torch.optim.RMSprop``
(lr 6.25e-5, alpha 0.95, eps 1.5e-7).  Here that learner is driven on EXACTLY the index /
IS-weight stream the HIP learner sampled (same replay, same transitions) for 200 steps and
the learners are compared step by step with an fp64 PyTorch learner on the same stream:
loss, priorities and the parameter trajectory.  The
reference ships no learning fixtures, so this pins self-consistency with the in-repo
PyTorch reference of the same algorithm ("parity unpinned" against upstream numbers)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

STEPS = 200


def _run(cuda, dtype: str, B: int = 256, steps: int = STEPS, seed: int = 1122):
    """HIP learner (``dtype``) + fp32 and fp64 PyTorch reference learners on the HIP
    learner's sampled stream.  Returns per-step trajectories and parameter distances."""
    from apex_amd.algo.losses import compute_loss_device, update_parameters_ex
    from apex_amd.engine.apex import ApexEngine, EngineConfig
    from apex_amd.engine.learner import LearnerConfig
    from apex_amd.models.dqn import DuelingDQN

    lc = LearnerConfig(batch_size=B, forward="hip", dtype=dtype)
    cfg = EngineConfig(n_envs=64, replay_capacity=16384, threshold_size=8192, learner=lc, seed=seed)
    eng = ApexEngine(cfg, cuda)
    eng.fill()
    L, rp = eng.learner, eng.replay

    def clone(src, dt):
        m = DuelingDQN.from_shapes((4, 84, 84), cfg.n_actions).to(cuda)
        m.load_state_dict(src.state_dict())
        return m.to(dt)

    refs = {}
    for name, dt in (("t32", torch.float32), ("t64", torch.float64)):
        m, t = clone(L.model, dt), clone(L.target, dt)
        for p in t.parameters():
            p.requires_grad_(False)
        opt = torch.optim.RMSprop(m.parameters(), lc.lr, alpha=lc.rms_alpha, eps=lc.rms_eps, centered=True)
        refs[name] = (m, t, opt, dt)
    p0 = L.flat.detach().double().clone()
    s = torch.empty(B, 4, 84, 84, dtype=torch.uint8, device=cuda)
    s2 = torch.empty_like(s)
    a = torch.empty(B, dtype=torch.int32, device=cuda)
    r = torch.empty(B, device=cuda)
    d = torch.empty(B, device=cuda)
    flat = lambda m: torch.cat([p.detach().double().reshape(-1) for p in m.parameters()])  # noqa: E731
    traj = []
    for i in range(steps):
        L.step()  # samples (idx, w) on device, 3 forwards, backward, clip, RMSprop, priority write
        rp.gather(L.idx, s, s2, a, r, d)
        row = {"hip_loss": float(L.loss.item()), "hip_prio": L.prio.double().clone()}
        for name, (m, t, opt, dt) in refs.items():
            batch = (s.to(dt), a.long(), r.to(dt), s2.to(dt), d.to(dt), L.w.to(dt))
            loss, prios = compute_loss_device(m, t, batch, lc.n_step, lc.gamma)
            update_parameters_ex(loss, m, opt, lc.max_norm)
            row[name + "_loss"] = float(loss.item())
            row[name + "_prio"] = prios.double()
        p64 = flat(refs["t64"][0])
        moved = float((p64 - p0).norm())
        row["moved"] = moved
        row["hip_vs_64"] = float((L.flat.double() - p64).norm()) / moved
        row["t32_vs_64"] = float((flat(refs["t32"][0]) - p64).norm()) / moved
        row["hip_vs_t32"] = float((L.flat.double() - flat(refs["t32"][0])).norm()) / moved
        row["param_rel"] = float((L.flat.double() - p64).norm() / p64.norm())
        row["t32_param_rel"] = float((flat(refs["t32"][0]) - p64).norm() / p64.norm())
        for k in ("hip", "t32"):
            row[k + "_prio_err"] = float(((row[k + "_prio"] - row["t64_prio"]).abs().max()
                                          / row["t64_prio"].abs().max()))
            row[k + "_loss_err"] = abs(row[k + "_loss"] - row["t64_loss"]) / max(abs(row["t64_loss"]), 1e-12)
        traj.append(row)
    return traj


def _summary(traj):
    keys = ("moved", "hip_vs_64", "t32_vs_64", "hip_vs_t32", "param_rel", "t32_param_rel", "hip_loss_err",
            "t32_loss_err", "hip_prio_err", "t32_prio_err")
    for i in (0, 1, 2, 5, 10, 25, 50, 100, len(traj) - 1):
        if i < len(traj):
            print(i, {k: f"{traj[i][k]:.3g}" for k in keys})


def test_first_step_distance_to_fp64_is_torch_fp32_class_over_seeds(cuda):
    """the step-0 update's distance to the fp64 learner's, as a fraction
    of the update length, for the HIP learner and for PyTorch's fp32 learner on the same
    batch, over 8 seeds (model init, replay contents and the sampled batch all change).  A
    single seed is the luck of one quadratic-region sample (see below); the median over seeds
    is the kernels' precision class.  Bound: HIP median <= 3x torch fp32's median (the round-3
    class), the worst seed within 3x torch's worst (table in profiles/r5_learning_first_step_seeds.md)."""
    rows = []
    for k in range(8):
        tr = _run(cuda, "fp32", steps=1, seed=1000 + 7 * k)
        rows.append((1000 + 7 * k, tr[0]["hip_vs_64"], tr[0]["t32_vs_64"], tr[0]["hip_loss_err"],
                     tr[0]["t32_loss_err"]))
    print("\n| seed | HIP vs fp64 | torch fp32 vs fp64 | HIP loss err | torch fp32 loss err |")
    print("|---:|---:|---:|---:|---:|")
    for r in rows:
        print(f"| {r[0]} | {r[1]:.3g} | {r[2]:.3g} | {r[3]:.3g} | {r[4]:.3g} |")
    med = lambda xs: sorted(xs)[len(xs) // 2]  # noqa: E731  (upper median of 8)
    hip, t32 = med([r[1] for r in rows]), med([r[2] for r in rows])
    print(f"median: HIP {hip:.3g}  torch fp32 {t32:.3g}  ratio {hip / t32:.2f}")
    assert hip <= 3.0 * t32, (hip, t32)
    # single seeds: either learner can land one quadratic-region sample's td on the wrong side of
    # a rounding (measured: torch fp32 2e-3 / 4e-3 on two of 8 seeds, HIP 3.7e-3 on another), so
    # the tails are compared, not the seeds one by one
    assert max(r[1] for r in rows) <= 3.0 * max(r[2] for r in rows), rows


def test_fp32_hip_learner_tracks_torch_fp32_learner(cuda):
    """Loss / priorities within ~2e-7 of fp64 from the first step.  The parameter distance of
    the first steps hinges on very few samples: with this random-init net on raw u8 frames
    |Q| ~ 100 and |td| ~ 12, so all but ~1 of the 256 samples sit in Huber's linear region
    (gradient +-w/B, exact); the one quadratic-region sample's td (a difference of two ~100
    values) carries all the rounding sensitivity.  Measured (MI355X, scripts/diag/grad_check.py):
    every activation as close to fp64 as PyTorch fp32's (conv1 output 4e-8 vs 2.5e-7, Q 6.2e-7
    vs 6.1e-7), that one td off by 2.9e-5 (torch fp32: 5.8e-6) -- both fp32 roundings of
    |Q| ~ 107 -- hence step-0 update distances to fp64 of 2.8e-4 (HIP) and 2.8e-5 (torch fp32)
    of the update length: the luck of one sample, so the first-step bound is on the distance
    to fp64, not on agreement with one fp32 rounding.  Beyond ~10 steps BOTH fp32 learners drift
    from the fp64 one at the same rate: the first centered-RMSprop steps are sign-like
    (update ~ lr * g / sqrt(var)), so roundoff-sized gradients of either sign move weights by
    a full lr -- an intrinsic property of the reference's algorithm, not of the kernels."""
    traj = _run(cuda, "fp32")
    _summary(traj)
    assert traj[-1]["moved"] > 0
    # first steps: loss and priorities at kernel precision (the multi-seed precision-class
    # bound on the update itself is the test above)
    # (multiplicative against torch fp32's own value on the same step -- measured, round 6:
    # HIP 1.2e-4 / 1.1e-4 / 1.4e-4 vs torch 2.8e-5 / 2.7e-5 / 2.5e-5; the 8-seed test above shows
    # which learner lands nearer fp64 is a per-seed coin toss)
    for row in traj[:3]:
        assert row["hip_vs_64"] <= 10.0 * row["t32_vs_64"], row
        assert row["hip_loss_err"] < 1e-4 and row["hip_prio_err"] < 1e-3
    # whole run: the HIP fp32 learner is no farther from the fp64 learner than PyTorch's
    # own fp32 learner (same fp32 roundoff class).  The sign-like RMSprop steps amplify any
    # roundoff difference chaotically from step ~3 on, and the torch fp32 reference is NOT
    # run-to-run deterministic (its conv backward): three runs of this seed in one process
    # (scripts/diag/learning_determinism.py, MI355X) gave the HIP learner 0.0681 at step 10
    # every time (bit-identical trajectory) and torch fp32 0.057 / 0.0029 / 4.3e-5 -- the
    # step at which torch's copy leaves fp64 is a coin toss, so steps of the divergence onset
    # are not compared one by one (a per-step bound there passed or failed with torch's luck).
    # Once both have saturated (the second half) every step is compared, and the tail means.
    # Every bound is multiplicative against torch fp32's own tail (no additive floors; measured,
    # round 6, steps 100 / 199: distance to fp64 HIP 0.60 / 0.74 vs torch 0.60 / 0.70, loss error
    # 0.019 / 0.045 vs 0.12 / 0.25, priority error 0.080 / 0.086 vs 0.13 / 0.076).
    tail = traj[len(traj) // 2:]
    mean = lambda k: sum(r[k] for r in tail) / len(tail)  # noqa: E731
    med = lambda k: sorted(r[k] for r in tail)[len(tail) // 2]  # noqa: E731
    for row in tail:
        assert row["hip_vs_64"] <= 1.5 * med("t32_vs_64"), row
        assert row["param_rel"] <= 3.0 * med("t32_param_rel"), row
    assert mean("hip_vs_64") <= 1.5 * mean("t32_vs_64")
    assert mean("param_rel") <= 2.0 * mean("t32_param_rel")
    assert mean("hip_loss_err") <= 3.0 * mean("t32_loss_err")
    assert mean("hip_prio_err") <= 2.0 * mean("t32_prio_err")


def test_bf16_hip_learner_stays_in_band(cuda):
    """The opt-in bf16 learner on the same stream: losses and priorities stay within a
    stated band of the fp64 PyTorch learner (bf16 operands: ~3 significant digits)."""
    traj = _run(cuda, "bf16")
    _summary(traj)
    # measured: step-1 loss 1.1e-3 / priorities 1.2e-2 from fp64; bf16 roundoff moves the
    # parameters off the fp64 trajectory earlier than fp32 does (0.64% vs 0.03% at ~step 20)
    # and both end within ~3% of it after 200 steps (fp32 2.7%, bf16 2.8-3.0%)
    assert traj[0]["hip_loss_err"] < 1e-2
    for row in traj:
        assert row["param_rel"] <= 2.0 * row["t32_param_rel"] + 0.02, row
    tail = traj[len(traj) // 2:]
    assert sum(r["hip_loss_err"] for r in tail) / len(tail) < 0.5
