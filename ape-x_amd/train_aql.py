"""GPU AQL training CLI (BASELINE config 4): ``python -m apex_amd.train_aql [flags]``.

The MI355X counterpart of the reference's multi-worker AQL trainer (AQL_dis.py:18-170 with
batchrecoder_AQL.py): instead of 10 forked CPU workers that each play one episode per
iteration and a learner that pickles weights to them, one :class:`AQLEngine` keeps E
vectorised GPU envs, the HBM prioritized replay with candidate sets and the fused learner
on one GPU (see ``apex_amd.engine.aql``).  One *iteration* = one step of all E envs + the
reference replay ratio of ``E // batch_size`` SGD steps (AQL_dis.py:118) + a weight
publish to the actors (AQL_dis.py:115).

Reference cadences and artefacts kept:

* target sync after iteration ``it`` when ``it % target_update_interval == 0`` (20;
  iteration 0 included, AQL_dis.py:127-129);
* ``model{it}.pth`` every ``save_interval`` (200) iterations and at the last one
  (AQL_dis.py:131-133, 136-137) -- the reference state_dict (``q.*`` / ``proposal.*`` keys,
  NoisyNet epsilon buffers included), loadable by the reference ``load_model`` -- plus a
  ``.train.pt`` sidecar (Adam moments, step counter, target net, iteration counters):
  ``--resume IT`` restores the optimizer state and counters, not weights only; the replay,
  the env states and the acting RNG counters are not saved, so training continues on a
  freshly filled replay (it does not replay the uninterrupted run bit for bit);
* tags ``learner/loss_q`` / ``learner/loss_proposal`` (means over the logging window, at
  the learner-step index; AQL_dis.py:123-124) and ``actor/episode_reward`` /
  ``actor/episode_length`` (batchrecoder_AQL.py:118-119), plus ``evaluator/episode_reward``
  from greedy episodes (the reference's ``training=False`` branch: ``q.eval()``, eps 0,
  AQL_dis.py:151-167) and ``learner/steps_per_sec`` / ``actor/env_steps_per_sec``.

Losses are accumulated on the device (no host sync per learner step); the host reads
them once per ``--log-interval`` iterations.

``--gpus N`` (N > 1; or any launch with WORLD_SIZE > 1): the distributed form of AQL_dis
across GPUs (``apex_amd.engine.central_aql``): rank 0 trains and checkpoints, ranks 1..N-1
are actor GPUs pushing transitions over HIP IPC; one iteration = one packet per actor +
``(N-1) * n_envs // batch_size`` SGD steps.  ``--same-device`` puts every rank on cuda:0
(rehearsal on one GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np
import torch

from . import envs
from .engine.aql import AQLEngine, AQLEngineConfig
from .models.aql import AQL
from .utils.checkpoint import load_model, load_train_state, save_model, save_train_state
from .utils.tb import NullWriter, SummaryWriter


def parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="AQL_dis on MI355X (GPU-resident AQL engine)")
    p.add_argument("--env", default="CartPole-v0", help="CartPole-v0/v1, Pendulum-v0/v1, BipedalWalker-v3")
    p.add_argument("--max-step", type=int, default=1_000_000, help="iterations (AQL_dis max_step)")
    p.add_argument("--n-envs", type=int, default=256, help="GPU envs (the reference's workers)")
    p.add_argument("--batch-size", type=int, default=32)
    p.add_argument("--gamma", type=float, default=0.99)
    p.add_argument("--n-steps", type=int, default=1)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--ent-lam", type=float, default=0.8)
    p.add_argument("--propose-sample", type=int, default=1)
    p.add_argument("--uniform-sample", type=int, default=50)
    p.add_argument("--action-var", type=float, default=0.25)
    p.add_argument("--prior-alpha", type=float, default=0.6)
    p.add_argument("--prior-beta-start", type=float, default=0.4)
    p.add_argument("--capacity", type=int, default=10_000_000, help="replay capacity (AQL_dis.py:44: 1e7)")
    p.add_argument("--target-update-interval", type=int, default=20, help="iterations (0 = off)")
    p.add_argument("--target-update-steps", type=int, default=0,
                   help="> 0: sync the target every this many learner steps instead (not the reference's cadence)")
    p.add_argument("--save-interval", type=int, default=200, help="iterations")
    p.add_argument("--save-dir", default=".")
    p.add_argument("--resume", default=None, help="iteration index of model{IDX}.pth in --save-dir, or 'latest'")
    p.add_argument("--log-dir", default=None, help="event-file directory (default runs/<time>-<env>-learner)")
    p.add_argument("--no-tb", action="store_true")
    p.add_argument("--log-interval", type=int, default=20, help="iterations between metric reads (host syncs)")
    p.add_argument("--eval-interval", type=int, default=0, help="iterations between greedy evaluations (0 = off)")
    p.add_argument("--eval-episodes", type=int, default=10)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--device", default="cuda:0")
    p.add_argument("--no-graphs", action="store_true")
    p.add_argument("--overlap", action="store_true",
                   help="acting on its own HIP stream beside the learner steps (the learner sees each acting "
                        "step's transitions one iteration later; a checkpoint does not hold the staged half)")
    p.add_argument("--json-log", default=None, help="append one JSON record per log interval to this file")
    p.add_argument("--gpus", type=int, default=1, help="N > 1: rank 0 learner + N-1 actor GPUs over HIP IPC")
    p.add_argument("--same-device", action="store_true", help="--gpus N on one GPU (every rank on cuda:0)")
    p.add_argument("--backend", default="gloo", choices=["gloo", "nccl"],
                   help="control-plane backend of the multi-rank form (the data plane is HIP IPC)")
    p.add_argument("--transport", default="auto", choices=["auto", "ipc", "p2p"],
                   help="the multi-rank form's experience links: HIP IPC rings, or torch.distributed p2p "
                        "(auto: IPC on GPUs)")
    p.add_argument("--launch-timeout", type=float, default=3600.0, help="--gpus N self-launch wall limit")
    return p


def config_from_args(a) -> AQLEngineConfig:
    return AQLEngineConfig(env_id=a.env, n_envs=a.n_envs, capacity=a.capacity, batch_size=a.batch_size,
                           gamma=a.gamma, n_steps=a.n_steps, lr=a.lr, ent_lam=a.ent_lam,
                           propose_sample=a.propose_sample, uniform_sample=a.uniform_sample,
                           action_var=a.action_var, alpha=a.prior_alpha, beta_start=a.prior_beta_start,
                           max_step=a.max_step, target_update_interval=a.target_update_interval,
                           target_update_steps=a.target_update_steps, track_losses=True,
                           use_graphs=not a.no_graphs, seed=a.seed, overlap=a.overlap)


# ------------------------------------------------------------------ checkpoint
def model_path(save_dir: str, idx: int) -> str:
    return os.path.join(save_dir, f"model{idx}.pth")


def save_engine(eng: AQLEngine, path: str) -> str:
    """model{it}.pth (reference keys; the online net incl. its noise buffers) + sidecar."""
    torch.cuda.synchronize(eng.device)
    L = eng.learner
    save_train_state(path, target=eng.target,
                     counters={"iteration": eng.iterations, "learner_steps": eng.learner_steps},
                     extra_tensors={"adam_m": L.m, "adam_v": L.v, "step_ctr": L.step_ctr})
    save_model(eng.model, path)
    return path


def load_engine(eng: AQLEngine, path: str, idx: int) -> dict:
    """Weights into the engine's flat buffers (parameters are views), then the sidecar if
    present (Adam moments, step counter, target net, counters); effective NoisyNet weights
    are recomputed and the actors get the loaded weights.  Training continues at
    iteration ``idx + 1`` (the file was written after iteration ``idx``)."""
    load_model(eng.model, path)
    L = eng.learner
    counters = {}
    if os.path.exists(path + ".train.pt"):
        st = load_train_state(path, target=eng.target, restore_rng=False)
        L.m.copy_(st["extra"]["adam_m"])
        L.v.copy_(st["extra"]["adam_v"])
        L.step_ctr.copy_(st["extra"]["step_ctr"])
        counters = st["counters"]
    else:
        eng.target.load_state_dict(eng.model.state_dict())
    eng.iterations = int(counters.get("iteration", idx + 1))
    eng.learner_steps = int(counters.get("learner_steps", 0))
    L.refresh()
    eng.publish()
    torch.cuda.synchronize(eng.device)
    return counters


def latest_index(save_dir: str) -> int | None:
    idx = []
    for f in os.listdir(save_dir) if os.path.isdir(save_dir) else []:
        if f.startswith("model") and f.endswith(".pth") and f[5:-4].isdigit():
            idx.append(int(f[5:-4]))
    return max(idx) if idx else None


# ------------------------------------------------------------------ evaluation
def greedy_eval(eng: AQLEngine, episodes: int, seed: int = 12345) -> list[float]:
    """The reference's evaluation branch (AQL_dis.py:151-167): a CPU copy of the online
    network with ``q.eval()`` (NoisyNet means), eps 0, env action ``a_mu[0][a]``."""
    env = envs.make(eng.cfg.env_id)
    env.seed(seed)
    cfg = eng.cfg
    m = AQL(env, propose_sample=cfg.propose_sample, uniform_sample=cfg.uniform_sample,
            action_var=cfg.action_var, device="cpu")
    torch.cuda.synchronize(eng.device)
    m.load_state_dict({k: v.detach().cpu() for k, v in eng.model.state_dict().items()})
    m.q.eval()
    out = []
    limit = int(getattr(env, "_max_episode_steps", None) or 10_000)
    for _ in range(episodes):
        s, er = env.reset(), 0.0
        for _ in range(limit):
            a, a_mu, _ = m.act(s, 0.0)
            s, r, d, _ = env.step(a_mu[0][a])
            er += float(r)
            if d:
                break
        out.append(er)
    env.close()
    return out


# ------------------------------------------------------------------ main
def train(a) -> dict:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and world == 1:  # self-launch one process per rank (never exec from a GPU process)
        import sys

        from .parallel.spawn import run_ranks

        code = run_ranks([sys.executable, "-m", "apex_amd.train_aql", *sys.argv[1:]], a.gpus, timeout=a.launch_timeout)
        if code:
            raise SystemExit(code)
        return {}
    if world > 1:
        return train_central(a, int(os.environ["RANK"]), world)
    dev = torch.device(a.device)
    torch.cuda.set_device(dev)
    eng = AQLEngine(config_from_args(a), dev)
    start = 0
    if a.resume is not None:
        idx = latest_index(a.save_dir) if a.resume == "latest" else int(a.resume)
        if idx is None:
            raise SystemExit(f"--resume latest: no model*.pth in {a.save_dir}")
        counters = load_engine(eng, model_path(a.save_dir, idx), idx)
        start = eng.iterations
        print(f"resumed from {model_path(a.save_dir, idx)} at iteration {start} {counters}", flush=True)
    writer = NullWriter() if a.no_tb else SummaryWriter(a.log_dir, comment=f"-{a.env}-learner")
    eng.fill()
    if not a.no_graphs:
        eng.capture()
    return _loop(a, eng, eng.iteration, eng.E, eng.finished_episodes, start, writer)


def train_central(a, rank: int, world: int) -> dict:
    """Rank 0: the AQL learner loop (logging, evaluation, checkpoints) over a
    :class:`CentralAQLEngine`; ranks 1..: act and push until rank 0 stops them."""
    import torch.distributed as dist

    from .engine.central_aql import CentralAQLEngine

    local = 0 if a.same_device else int(os.environ.get("LOCAL_RANK", rank))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if a.backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    ceng = CentralAQLEngine(config_from_args(a), dev, rank, world, transport=a.transport)
    last = {}
    try:
        if rank != 0:
            if not a.no_graphs:
                ceng.capture()
            while ceng.iteration():
                pass
            torch.cuda.synchronize(dev)
            return {}
        if a.resume is not None:
            idx = latest_index(a.save_dir) if a.resume == "latest" else int(a.resume)
            if idx is None:
                raise SystemExit(f"--resume latest: no model*.pth in {a.save_dir}")
            load_engine(ceng.eng, model_path(a.save_dir, idx), idx)
            ceng.restore(ceng.eng.iterations, ceng.eng.learner_steps)
        writer = NullWriter() if a.no_tb else SummaryWriter(a.log_dir, comment=f"-{a.env}-learner-central")
        ceng.fill()
        if not a.no_graphs:
            ceng.capture()
        last = _loop(a, ceng.eng, ceng.iteration, ceng.R * ceng.E, lambda: [], ceng.iterations, writer,
                     central=ceng)
        last["links"] = ceng.close()
        print(json.dumps({"links": last["links"]}), flush=True)
    finally:
        if rank == 0:
            ceng.close()
        dist.destroy_process_group()
    return last


def _crossed(lo: int, hi: int, every: int, offset: int = 0) -> bool:
    """Some k in [lo, hi] with (k + offset) % every == 0."""
    if hi < lo or every <= 0:
        return False
    return (hi + offset) // every * every >= lo + offset


def _loop(a, eng: AQLEngine, iterate, envs_per_iter: int, episodes, start: int, writer, central=None) -> dict:
    """The training loop: ``iterate()`` per iteration (act + K SGD steps + publish + target
    cadence, or its central form), checkpoints, metrics and greedy evaluations.

    Central: one ``iterate()`` is a learner SPIN (ingest + the SGD steps the applied rows
    pay for); the iteration count, checkpoint / log / eval cadences and ``max_step`` follow
    the recorded batches that reached the replay (CentralAQLEngine.data_iterations), and the
    logged step counts / rates read the device SGD counter (one sync per log window)."""
    ep_idx, last = 0, {}
    t_win, it_win, steps_win = time.perf_counter(), start, eng.learner_steps
    jl = open(a.json_log, "a") if a.json_log else None
    it = start  # the next iteration to complete
    try:
        while it < a.max_step:
            iterate()   # act + K SGD steps + publish + (it % 20 == 0) target sync
            if central is not None:
                done = min(central.iterations, a.max_step)  # iterations completed so far
                if done <= it:
                    continue  # a spin that completed no recorded batch
                lo, hi = it, done - 1
                eng.iterations = done
            else:
                lo = hi = it
            it = hi + 1
            if _crossed(lo, hi, a.save_interval) or hi == a.max_step - 1:
                if central is not None:
                    central.refresh_steps()
                save_engine(eng, model_path(a.save_dir, hi))
            log_now = _crossed(lo, hi, a.log_interval, 1 - start) or hi == a.max_step - 1
            ev = a.eval_interval > 0 and (_crossed(lo, hi, a.eval_interval, 1) or hi == a.max_step - 1)
            if not (log_now or ev):
                continue
            if central is not None:
                central.refresh_steps()
            lq, lp, n = eng.learner.take_loss_means()
            eps = episodes()
            now = time.perf_counter()
            dt = max(now - t_win, 1e-9)
            if n:
                writer.add_scalar("learner/loss_q", lq, eng.learner_steps)
                writer.add_scalar("learner/loss_proposal", lp, eng.learner_steps)
            for r, length in eps:
                writer.add_scalar("actor/episode_reward", r, ep_idx)
                writer.add_scalar("actor/episode_length", length, ep_idx)
                ep_idx += 1
            sps = (eng.learner_steps - steps_win) / dt
            writer.add_scalar("learner/steps_per_sec", sps, eng.learner_steps)
            writer.add_scalar("actor/env_steps_per_sec", (hi + 1 - it_win) * envs_per_iter / dt, eng.learner_steps)
            last = {"iteration": hi, "learner_steps": eng.learner_steps, "loss_q": lq, "loss_proposal": lp,
                    "episodes": len(eps), "actor_mean_return": float(np.mean([r for r, _ in eps])) if eps else None,
                    "sgd_steps_per_s": round(sps, 1), "target_syncs": len(eng.target_syncs)}
            if central is not None:
                last["packets_applied"] = sum(central.applied.values())
                last["learner_spins"] = central.spins
            if ev:
                ret = greedy_eval(eng, a.eval_episodes, seed=a.seed + 7 * hi)
                for k, r in enumerate(ret):
                    writer.add_scalar("evaluator/episode_reward", r, eng.learner_steps)
                last["greedy_mean_return"] = float(np.mean(ret))
            print(json.dumps(last), flush=True)
            if jl:
                jl.write(json.dumps(last) + "\n")
                jl.flush()
            t_win, it_win, steps_win = time.perf_counter(), hi + 1, eng.learner_steps
    finally:
        writer.flush()
        if jl:
            jl.close()
    return last


def main(argv=None) -> int:
    train(parser().parse_args(argv))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
