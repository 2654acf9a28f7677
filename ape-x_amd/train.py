"""GPU-resident Ape-X training CLI: ``python -m apex_amd.train [arguments.py flags]``.

The production entry point for the MI355X engine (one process per GPU).  It replaces
the reference's replay.py + learner.py + N x actor.py deployment with
one rank per GPU, launched directly (1 GPU) or under ``torch.distributed.run`` (any
number of GPUs and nodes; RCCL over xGMI inside a node):

* ``--topology central`` (default for N > 1, ``config.py``): rank 0 is THE learner with the
  one replay (the reference's single learner, origin_repo/learner.py:134-175); ranks 1..
  are actor GPUs pushing experience into rank 0's HBM over HIP IPC rings (xGMI peer
  copies, ``apex_amd.parallel.ipc``).  A multi-GPU preflight runs first: if peer access
  or the IPC round trip fails, the experience links fall back to torch.distributed
  send/recv (RCCL, ``apex_amd.parallel.experience``) instead of failing the job.
* ``--topology sharded``: every rank runs an actor shard, its HBM replay shard and a
  data-parallel learner replica; gradients are all-reduced over RCCL and the shards are
  sampled as one global prioritized buffer (``apex_amd.parallel.sharded``).

Reference cadences and tags are kept: target sync every ``--target_update_interval``
(learner.py:163-165), weights published every ``--publish_param_interval``
(learner.py:169-170), ``model.pth`` written every ``--save_interval`` (learner.py:166-168)
plus a ``model.pth.train.pt`` sidecar (optimizer moments, step counters, target net)
for a true resume (``--resume``), ``learner/loss``, ``learner/grad_norm``,
``learner/BPS`` every ``--bps_interval`` (learner.py:151-175), ``actor/episode_reward``
and ``actor/episode_length`` (actor.py:91-92), plus ``learner/steps_per_sec``,
``actor/frames_per_sec`` and ``replay/size``.  The envs are the GPU
synthetic Atari-shaped envs of ``ActorShard`` (no emulator in this image).
"""
from __future__ import annotations

import os
import sys
import time

import torch
import torch.distributed as dist

from .config import args_to_config, build_parser, preset
from .utils.checkpoint import save_model, sidecar_path


def parser():
    p = build_parser(preset("origin"), description="Ape-X DQN on MI355X (GPU-resident engine)")
    p.add_argument("--actions", type=int, default=18, help="action count of the synthetic env (Seaquest: 18)")
    p.add_argument("--actor-steps", type=int, default=1, help="actor steps per learner step")
    p.add_argument("--save-path", default="model.pth")
    p.add_argument("--resume", default=None, help="model.pth (+ .train.pt sidecar) to resume from")
    p.add_argument("--log-dir", default=None, help="event-file directory (default runs/<time>-<env>-learner)")
    p.add_argument("--no-tb", action="store_true")
    p.add_argument("--same-device", action="store_true", help="all ranks on cuda:0 (1-GPU rehearsal with gloo)")
    p.add_argument("--eval-envs", type=int, default=8,
                   help="greedy evaluator envs on rank 0 (eps 0, unclipped rewards, origin_repo/eval.py); 0 = off")
    p.add_argument("--eval-interval", type=int, default=50, help="learner steps between evaluator chunks")
    p.add_argument("--eval-steps", default="25",
                   help="evaluator env steps per chunk, or 'auto': enough that every evaluator env can finish a "
                        "capped episode (max_episode_length steps) inside each log window of --bps_interval "
                        "learner steps (run as captured graphs of 100 steps; slows training wall-clock, not "
                        "its per-step dynamics)")
    return p


# ------------------------------------------------------------------ checkpoint
def _weights_tag(flat: torch.Tensor) -> torch.Tensor:
    """Cheap fingerprint of the model weights (fp64 sum, sum of squares, a strided sample)
    stored in the sidecar: ``load_engine`` only restores optimizer moments / counters that
    belong to the model file it loaded."""
    f = flat.detach().double().cpu()
    return torch.cat([f.sum().view(1), f.pow(2).sum().view(1), f[:: max(1, f.numel() // 61)][:61]])


def _learner_state(learner, counters: dict) -> dict:
    return {"opt_s1": learner.opt_s1.cpu(), "opt_s2": learner.opt_s2.cpu(),
            "step_counter": learner.step_counter.cpu(), "target_flat": learner.tflat.cpu(),
            "counters": dict(counters), "weights_tag": _weights_tag(learner.flat)}


def save_engine(learner, path: str, counters: dict) -> None:
    """model.pth (the reference state_dict: enjoy.py / load_model read it) + sidecar.  The
    sidecar goes first, through tmp + os.replace like the model file, and carries a
    fingerprint of the weights: a kill between the two writes leaves a sidecar that
    ``load_engine`` recognises as belonging to a different model file."""
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    side = sidecar_path(path)
    torch.save(_learner_state(learner, counters), side + ".tmp")
    os.replace(side + ".tmp", side)
    save_model(learner.model, path)


def load_engine(learner, path: str) -> dict:
    """Load weights (+ sidecar if present) into a DQNLearner; returns the counters."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    learner.model.load_state_dict(sd)   # parameters are views of the flat buffer
    counters = {}
    side = sidecar_path(path)
    st = torch.load(side, map_location="cpu", weights_only=True) if os.path.exists(side) else None
    if st is not None and "weights_tag" in st and not torch.allclose(st["weights_tag"], _weights_tag(learner.flat),
                                                                     rtol=1e-9, atol=0.0):
        import warnings

        warnings.warn(f"{side} does not belong to {path} (torn save?): resuming weights only")
        st = None
    if st is not None:
        learner.opt_s1.copy_(st["opt_s1"])
        learner.opt_s2.copy_(st["opt_s2"])
        learner.step_counter.copy_(st["step_counter"])
        learner.tflat.copy_(st["target_flat"])
        counters = dict(st.get("counters", {}))
    else:
        learner.tflat.copy_(learner.flat)
    if getattr(learner, "hip_net", False):
        learner.refresh_packed()
        learner.tnet.repack()
    return counters


# ------------------------------------------------------------------ main
def main(argv=None) -> int:
    args = parser().parse_args(argv)
    cfg = args_to_config(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    from .utils import trace

    if cfg.kernel.hip_debug:  # before the HIP runtime starts
        trace.hip_debug_env(cfg.kernel.hip_debug)
    if cfg.kernel.profile:
        trace.enable(True)
    if not torch.cuda.is_available():
        raise SystemExit("apex_amd.train runs the GPU engine; use apex_amd.trainers.* or the roles on CPU")
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    backend = cfg.dist.backend if cfg.dist.backend != "auto" else "nccl"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": device} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    topology = cfg.replay.topology if world > 1 else "single"
    transport = "auto"
    if topology == "central":  # prove the cross-device paths; IPC -> p2p fallback (parallel/preflight.py)
        from .parallel import preflight

        rep = preflight.run(device, ipc=True, timeout=90.0, fallback=True)
        transport = rep["transport"]
        if rep.get("transport_fallback") and rank == 0:
            print(f"preflight: IPC experience links unavailable ({rep['transport_fallback']}); using p2p links",
                  file=sys.stderr)

    from .engine.apex import ApexEngine, EngineConfig
    from .engine.learner import LearnerConfig

    L, R = cfg.learner, cfg.replay
    lc = LearnerConfig(batch_size=R.batch_size, n_step=cfg.n_steps, gamma=cfg.gamma, lr=L.lr, rms_alpha=L.rms_alpha,
                       rms_eps=L.rms_eps, centered=L.centered, max_norm=L.max_norm, lr_gamma=L.lr_gamma,
                       lr_step_size=L.lr_step_size, beta=R.beta, optimizer=L.optimizer, forward=cfg.kernel.forward,
                       dtype=cfg.kernel.dtype,
                       seed=cfg.seed + (rank if topology == "sharded" else 0))
    E = cfg.actor.n_envs
    ecfg = EngineConfig(n_envs=E, n_actions=args.actions, replay_capacity=R.replay_buffer_size, alpha=R.alpha,
                        threshold_size=R.threshold_size, actor_steps_per_learner_step=args.actor_steps,
                        publish_param_interval=L.publish_param_interval,
                        target_update_interval=L.target_update_interval, nstep_mode=cfg.actor.nstep_mode,
                        eps_base=cfg.actor.eps_base, eps_alpha=cfg.actor.eps_alpha, exact_mass=R.exact_mass,
                        use_graphs=cfg.kernel.use_graphs, seed=cfg.seed, learner=lc)
    counters = {}
    if topology == "central":
        from .engine.central import CentralApexEngine

        eng = CentralApexEngine(ecfg, device, rank, world, transport=transport)
        learner = eng.learner if rank == 0 else None
        if args.resume and rank == 0:
            counters = load_engine(learner, args.resume)
        if args.resume:
            eng.publish_params()  # rank 0: a new parameter version on every link
        n_actor_gpus = world - 1
    else:
        from .parallel.dp import FlatGradAllReduce

        ecfg.actor_offset, ecfg.total_actors = rank * E, world * E
        ecfg.seed = cfg.seed + 7919 * rank
        allreduce = None
        if world > 1 and backend == "nccl":  # per-step gradients on a direct RCCL communicator
            from .parallel.rccl import RcclGradAllReduce

            try:
                allreduce = RcclGradAllReduce(device)
            except RuntimeError as e:
                print(f"rank {rank}: direct RCCL unavailable ({e}); torch.distributed collectives", flush=True)
        if world > 1 and allreduce is None:
            allreduce = FlatGradAllReduce(world)
        from .parallel.rccl import RcclGradAllReduce

        ecfg.overlap = True
        ecfg.dp_graph = isinstance(allreduce, RcclGradAllReduce)  # all-reduces captured in the learner graph
        eng = ApexEngine(ecfg, device, allreduce=allreduce, sharded=world > 1)
        learner = eng.learner
        if args.resume:
            counters = load_engine(learner, args.resume)
        if world > 1:
            from .parallel.broadcast import broadcast_flat

            broadcast_flat(learner.flat, src=0)
            broadcast_flat(learner.tflat, src=0)
            learner.refresh_packed()
            if learner.hip_net:
                learner.tnet.repack()
        eng.publish_params()
        n_actor_gpus = world
    start = int(counters.get("learn_steps", 0))
    eng.learn_steps = start

    writer = None
    if rank == 0 and not args.no_tb:
        from .utils.tb import SummaryWriter

        writer = SummaryWriter(args.log_dir, comment=f"-{cfg.env.env}-learner")
    t_fill = time.perf_counter()
    eng.fill()
    if cfg.kernel.use_graphs:
        eng.capture()
    torch.cuda.synchronize(device)
    if rank == 0:
        print(f"replay warm ({time.perf_counter() - t_fill:.1f}s); training from step {start}", flush=True)

    evaluator = None
    if rank == 0 and args.eval_envs > 0:
        from .engine.evaluator import GPUEvaluator

        src_model = eng.actor_model if hasattr(eng, "actor_model") else learner.model
        evaluator = GPUEvaluator(src_model, args.eval_envs, args.actions, forward=cfg.kernel.forward,
                                 dtype=cfg.kernel.dtype, device=device, seed=cfg.seed + 31337,
                                 episode_life=bool(cfg.env.episode_life), max_episode_steps=cfg.env.max_episode_length)
        eval_stream = torch.cuda.Stream(device=device)
        ev_loaded = torch.cuda.Event()
        if str(args.eval_steps) == "auto":
            chunks = max(1, L.bps_interval // max(1, args.eval_interval))
            eval_steps = -(-int(cfg.env.max_episode_length) // chunks)
        else:
            eval_steps = int(args.eval_steps)
        if cfg.kernel.use_graphs and eval_steps >= 100:
            with torch.cuda.stream(eval_stream):
                evaluator.capture(100)
            torch.cuda.synchronize(device)
        print(f"evaluator: {args.eval_envs} envs, {eval_steps} greedy steps per {args.eval_interval} learner steps "
              f"(episode cap {int(cfg.env.max_episode_length)})", flush=True)

    def eval_chunk():
        """Latest published weights -> evaluator (ordered after the publish on the training
        stream, which in turn waits only for the copy), then greedy steps on the side stream."""
        cur = torch.cuda.current_stream(device)
        eval_stream.wait_stream(cur)
        with torch.cuda.stream(eval_stream):
            if hasattr(eng, "actor_flat"):
                evaluator.load(eng.actor_flat, getattr(eng, "actor_net", None))
            else:
                evaluator.load(learner.flat, getattr(learner, "net", None))
            ev_loaded.record(eval_stream)
            evaluator.run(eval_steps)
        cur.wait_event(ev_loaded)

    max_step = int(L.max_step)
    bps_every = max(1, L.bps_interval)
    frames_per_round = n_actor_gpus * args.actor_steps * eng.frames_per_actor_step
    step = eng.learn_steps  # capture's warm-up steps are real training steps
    t_last, step_last = time.perf_counter(), step
    eval_rets, eval_lens = [], []
    while not max_step or step < max_step:
        if eng.train_step() is False:  # central actor rank: the learner stopped this link
            break
        step = eng.learn_steps
        if evaluator is not None and step % max(1, args.eval_interval) == 0:
            eval_chunk()
        if learner is not None and step % bps_every == 0:
            torch.cuda.synchronize(device)
            now = time.perf_counter()
            dt_log = now - t_last
            sps = (step - step_last) / dt_log
            t_last, step_last = now, step
            if topology == "central" and rank == 0:  # async links: frames that actually reached the replay
                applied = sum(eng.applied.values())
                fps_measured = (applied - getattr(eng, "_applied_last", 0)) * eng.frames_per_actor_step / dt_log
                eng._applied_last = applied
            if learner is not None and rank == 0:
                st = learner.stats()
                # sharded DP: one synchronous update per step over a global batch of B * world, so
                # updates/s = sps and batches of B sampled per second = sps * world
                line = {"learner/loss": st["loss"], "learner/grad_norm": st["grad_norm"],
                        "learner/grad_norm_l2": st["grad_norm_l2"], "learner/BPS": sps,
                        "learner/updates_per_sec": sps,
                        "learner/batches_per_sec": sps * (world if topology == "sharded" else 1),
                        "actor/frames_per_sec": (fps_measured if topology == "central"
                                                 else sps * frames_per_round)}
                if evaluator is not None:
                    for r, n in evaluator.poll():
                        eval_rets.append(r)
                        eval_lens.append(n)
                    if eval_rets:  # episodes finished since the last log line
                        line["evaluator/episode_reward"] = sum(eval_rets) / len(eval_rets)
                        line["evaluator/episode_length"] = sum(eval_lens) / len(eval_lens)
                        line["evaluator/episodes"] = float(evaluator.episodes)
                        # episodes that ended at the step cap (eval.py:77's max_episode_length)
                        line["evaluator/capped_episodes"] = float(sum(n >= evaluator.max_episode_steps
                                                                      for n in eval_lens))
                        eval_rets, eval_lens = [], []
                    run_ret, run_len = evaluator.running()  # episodes still in progress
                    line["evaluator/running_return"] = float(run_ret.mean())
                    line["evaluator/running_length"] = float(run_len.mean())
                shard = getattr(eng, "actor", None)
                if shard is not None:
                    ret, length, count = shard.episode_stats()
                    done = count > 0
                    if bool(done.any()):
                        line["actor/episode_reward"] = float(ret[done].mean())
                        line["actor/episode_length"] = float(length[done].float().mean())
                line["replay/size"] = float(len(eng.replay))
                print(f"Step: {step} " + " ".join(f"{k}={v:.4g}" for k, v in line.items()), flush=True)
                if writer is not None:
                    for k, v in line.items():
                        writer.add_scalar(k, v, step)
        if L.save_interval and step % L.save_interval == 0 and rank == 0 and learner is not None:
            print("Saving Model..", flush=True)
            save_engine(learner, args.save_path, {"learn_steps": step, "actor_steps": eng.actor_steps})
    torch.cuda.synchronize(device)
    if rank == 0 and learner is not None:
        save_engine(learner, args.save_path, {"learn_steps": step, "actor_steps": eng.actor_steps})
    if writer is not None:
        writer.close()
    if topology == "central":  # async links: bounded stop handshake instead of a barrier
        if rank == 0:
            print(f"links: {eng.close()}", flush=True)
        dist.destroy_process_group()
    elif world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
