#!/usr/bin/env python
"""Headline benchmark: Ape-X DQN learner SGD steps/s + actor frames/s on MI355X.

Metric and config come from BASELINE.json: learner SGD steps/sec (+ actor frames/sec)
for Ape-X dueling double DQN on Atari-shaped 84x84x4 synthetic frames, batch 512,
n-step 3, PER alpha 0.6 / beta 0.4, centered RMSprop (lr 6.25e-5), grad clip 40,
target sync 2500, 18 actions (Seaquest, the reference's published run), random-init
weights.  The reference publishes 10-12 batches/s (its implementation, V100 learner)
and quotes 19 batches/s for the Ape-X paper (origin_repo/README.md:42).

Every rank (one per GPU) runs an actor shard (``--envs`` GPU envs with the global
Ape-X epsilon ladder), its HBM replay shard (``--capacity`` transitions) and a
learner replica; learner replicas are data-parallel (flat-gradient RCCL all-reduce)
and sample the shards as one global prioritized buffer (shard-mass all-gather,
``apex_amd.parallel.sharded``), so per-GPU work is fixed as N grows (weak scaling)
and the global batch is 512*N.
One timed step = one learner SGD step (sample 512 -> 3 forwards -> backward ->
clip -> RMSprop -> priority update) + ``--actor-steps`` actor steps of all envs.

``value`` = learner sample throughput in batches of 512 per second (sampled transitions/s
divided by 512: the unit of the reference's 10-12 batches/s).  With one GPU that is the
optimizer-update rate; under ``--scaling weak`` (data parallel, global batch 512*N) one
optimizer update consumes N such batches, so ``optimizer_updates_per_s`` (one synchronous
update per step) and ``learner_samples_per_sec`` are reported separately; ``--scaling
strong`` keeps the reference's single-learner global batch of 512 (512/N per rank), so
``value`` equals the update rate.  Actor frames/s (4 emulator frames per env step) is
reported alongside.  ``--dtype fp32`` (default) is the reference's precision
(origin_repo/learner.py:139-145: fp32 modules, no autocast): fp32 operands and activations,
the GEMMs on the bf16 matrix cores through an exact three-term split of every fp32 operand
(six products per 16 k, dropped terms below 2^-26 |a b|; per-layer error vs fp64 within the
fp32 dot-product bound, tests/test_gpu_f32_net.py::test_gemm_layers_are_fp32_class);
``--dtype bf16`` is the opt-in bf16-operand mode.  Run: ``python bench.py [--gpus N --steps K --warmup W]`` (N>1
under torch.distributed.run, one process per GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REFERENCE_BATCHES_PER_S = 12.0   # upper end of the reference's 10-12 batches/s
# central topology: transition rows rank 0 ingests per learner step, split over the actor GPUs
# (envs per actor GPU in CENTRAL_MIN_ENVS..2048, multiples of 64): the learner stays >= 95 % of
# the 1-GPU engine while the frames reaching the replay grow with N (emulated links, one MI355X,
# vs the 1-GPU engine's 2483 steps/s: R = 1 x 2048 envs 2556, R = 3 x 1344 2409, R = 7 x 640
# 2377 steps/s; profiles/r6_central_capacity.md)
CENTRAL_ROW_BUDGET = 4032
CENTRAL_MIN_ENVS = 640
PAPER_BATCHES_PER_S = 19.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=256, help="GPU envs (actors) per GPU")
    ap.add_argument("--actor-steps", type=int, default=1, help="actor steps per learner step (>= 1)")
    ap.add_argument("--batch", type=int, default=512, help="global batch at N=1 (per-rank batch under weak scaling)")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="learner/actor compute precision: fp32 = the reference's (fp32 MFMA kernels), bf16 = opt-in")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: batch per rank fixed (global batch batch*N); strong: global batch fixed (batch/N per rank)")
    ap.add_argument("--capacity", type=int, default=2_000_000)
    ap.add_argument("--threshold", type=int, default=50_000)
    ap.add_argument("--fill", action="store_true",
                    help="fill the whole replay (every transition slot written, frame ring wrapped to capacity) "
                         "before timing: BASELINE config 5 with --capacity 10000000")
    ap.add_argument("--actions", type=int, default=18)
    ap.add_argument("--forward", default="hip", choices=["torch", "hip"])
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--graph-warm", type=int, default=200,
                    help="real train steps replayed back to back right after graph capture, before the --warmup "
                         "steps (untimed, counted as training; ~0.1 s): the GPU reaches its sustained clock only "
                         "after a stretch of load, so a short timed window right after setup is not a ramp "
                         "measurement (20-step windows, one box: 2276-2318 steps/s after 48, 2310-2345 after "
                         "200, 2345 sustained over 2000 steps; profiles/archive_r5.md (r5_short_window.txt))")
    ap.add_argument("--tree-ride", type=int, default=1, choices=[0, 1],
                    help="1: the learner's priority-tree write rides the trunk backward's launches as extra "
                         "workgroups (no tree stream fork / join); 0: the forked tree stream")
    ap.add_argument("--draw-in-conv1", type=int, default=1, choices=[0, 1],
                    help="1: the learner's PER draw runs inside the conv1 forward launch; 0: its own sampling "
                         "launch at the chain head")
    ap.add_argument("--actor-at", default="start", choices=["start", "loss"],
                    help="overlapped engine: start the actor graph with the learner step, or after its fused "
                         "loss + heads backward (beside the trunk backward)")
    ap.add_argument("--no-overlap", dest="overlap", action="store_false",
                    help="run the actor graph after the learner step on the same stream (default: the actor "
                         "graph runs on its own HIP stream, concurrent with the learner step)")
    ap.add_argument("--seed", type=int, default=1122)
    ap.add_argument("--profile-steps", type=int, default=0, help="extra untimed steps after timing (for rocprof)")
    ap.add_argument("--no-reserve", dest="reserve", action="store_false",
                    help="do not take the actor stream from the pool before the process group")
    ap.add_argument("--roctx", action="store_true", help="roctx ranges around engine phases (rocprofv3 --marker-trace)")
    ap.add_argument("--topology", default="auto", choices=["auto", "central", "sharded"],
                    help="auto (default): one GPU = the single-GPU engine, N>1 = central (BASELINE config 3, the "
                         "reference's design: rank 0 = the one learner at batch 512 + the replay, ranks 1.. = actor "
                         "GPUs pushing experience over HIP IPC); sharded: a data-parallel learner per GPU sampling "
                         "the shards as one global PER (global batch 512*N; value = sample throughput / 512)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"], help="gloo: host-staged (tests)")
    ap.add_argument("--same-device", action="store_true", help="all ranks on cuda:0 (1-GPU rehearsal, gloo)")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "torch"],
                    help="data-parallel gradient all-reduce: direct RCCL communicator (default) or torch.distributed")
    ap.add_argument("--no-dp-graph", dest="dp_graph", action="store_false",
                    help="data-parallel: three phase graphs with eager RCCL all-reduces in between (default: the "
                         "all-reduces are captured inside ONE learner hipGraph per step; forced-DP 1-rank A/B 2615 -> "
                         "3050 steps/s)")
    ap.add_argument("--force-dp", action="store_true",
                    help="run the data-parallel step (RCCL collectives, sharded sampling) even with 1 rank "
                         "(under torch.distributed.run --nproc-per-node 1): measures its single-GPU overhead")
    ap.add_argument("--local-sampling", action="store_true",
                    help="N>1: sample each replay shard on its own (default: global PER over shards)")
    ap.add_argument("--algo", default="apex", choices=["apex", "aql"],
                    help="apex: the headline Ape-X DQN bench; aql: the GPU AQL engine (BASELINE config 4, "
                         "AQL_dis BipedalWalker-shaped; one step = one actor step of --envs envs + envs/32 SGD steps)")
    ap.add_argument("--aql-env", default="BipedalWalker-v3")
    ap.add_argument("--aql-overlap", action="store_true",
                    help="--algo aql: acting on its own HIP stream beside the learner steps (staged transitions)")
    ap.add_argument("--launch-timeout", type=float, default=560.0,
                    help="--gpus N>1 without torch.distributed.run: wall limit of the self-launched ranks "
                         "(inside the driver's 600 s)")
    ap.add_argument("--watchdog", type=float, default=240.0,
                    help="no-progress limit in seconds (0 = off): re-armed at every phase and every few hundred "
                         "steps; a rank that makes no progress for this long (a hung collective, IPC credit wait "
                         "or peer copy) dumps every thread's stack and exits 1, inside the driver's 600 s")
    ap.add_argument("--no-preflight", dest="preflight", action="store_false",
                    help="N>1: skip the multi-GPU preflight (peer access, IPC round trip, RCCL all-reduce)")
    ap.add_argument("--central-envs", default="auto",
                    help="central topology (N>1, --emulate-links): envs per actor GPU; each actor GPU pushes one "
                         "packet of this many transitions per learner step.  auto: rank 0's ingest budget of "
                         f"{CENTRAL_ROW_BUDGET} rows per learner step split over the N-1 actor GPUs (multiples of "
                         f"64, {CENTRAL_MIN_ENVS}..2048): the learner stays >= 95 %% of the 1-GPU engine while the frames "
                         "reaching the replay grow (profiles/r6_central_capacity.md)")
    ap.add_argument("--transport", default="auto", choices=["auto", "ipc", "p2p"],
                    help="central topology: HIP IPC rings in rank 0's HBM (auto on GPUs) or torch.distributed P2P links")
    ap.add_argument("--emulate-links", type=int, default=0, metavar="R",
                    help="one GPU: the central learner (rank 0) with R actor links emulated in-process (synthetic "
                         "packets into the real IPC ring, the real in-graph ingest): its load at N = R + 1 GPUs")
    ap.add_argument("--actor-only", default="", metavar="E,E,..",
                    help="one GPU: an actor rank's own throughput, unpaced (act + n-step rows + packet staging + the "
                         "packet copy), at each env count, e.g. 256,1024,4096")
    ap.add_argument("--unpaced", action="store_true",
                    help="central topology: actors run free (default: paced at --actor-steps packets per learner "
                         "step per actor through the credit window)")
    args = ap.parse_args()
    if args.actor_steps < 1:
        ap.error("--actor-steps must be >= 1 (the overlapped engine stages one actor step per learner step)")
    return args


def _host_launch_cost(eng, device, n: int = 20) -> float:
    """Median host time of one train_step enqueued into an idle GPU (extra, untimed steps)."""
    import statistics

    import torch

    lat = []
    for _ in range(n):
        torch.cuda.synchronize(device)
        t1 = time.perf_counter()
        eng.train_step()
        lat.append(time.perf_counter() - t1)
    torch.cuda.synchronize(device)
    return statistics.median(lat)


class Watchdog:
    """No-progress watchdog: ``kick()`` re-arms faulthandler's timer (stack dump of every
    thread, then exit 1) -- a long healthy run is never killed, a stall is."""

    def __init__(self, seconds: float):
        self.s = float(seconds)
        self._t = 0.0
        self.kick()

    def kick(self, every: float = 0.0) -> None:
        if self.s <= 0:
            return
        now = time.monotonic()
        if every and now - self._t < every:
            return
        self._t = now
        import faulthandler

        faulthandler.dump_traceback_later(self.s, exit=True)

    def off(self) -> None:
        if self.s > 0:
            import faulthandler

            faulthandler.cancel_dump_traceback_later()


def select_topology(topology: str, world: int) -> str:
    """auto: "single" for one rank, "central" (BASELINE config 3) for more."""
    if topology == "auto":
        return "central" if world > 1 else "single"
    if topology == "central" and world < 2:
        raise SystemExit("--topology central needs >= 2 ranks")
    return topology if world > 1 else "single"


def run_preflight(args, topo: str, device, wd: "Watchdog") -> dict | None:
    """N>1: prove peer access, the IPC round trip and the collective before timing."""
    if not args.preflight:
        return None
    from apex_amd.parallel import preflight

    ipc = topo == "central" and args.transport in ("auto", "ipc")
    rep = preflight.run(device, ipc=ipc, timeout=90.0, fallback=args.transport == "auto")
    wd.kick()
    return rep


def resolve_transport(requested: str, pre: dict | None) -> tuple[str, str | None]:
    """The central topology's experience transport after the preflight: ``auto`` takes the
    preflight's decision -- HIP IPC, or the torch.distributed p2p links (RCCL send/recv)
    with the reason when peer access or the IPC round trip failed.  An explicit choice
    stands (``ipc`` then fails in the preflight, by request)."""
    if requested != "auto" or not pre or "transport" not in pre:
        return requested, None
    return pre["transport"], pre.get("transport_fallback")


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # Not under torch.distributed.run: launch the N ranks here.  This process never
        # touches the GPU; the children are fresh processes (Popen, not exec) that re-enter
        # main() with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set; rank 0 prints the JSON line.
        from apex_amd.parallel.spawn import run_ranks

        sys.exit(run_ranks([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], args.gpus,
                           timeout=args.launch_timeout))
    wd = Watchdog(args.watchdog)
    import torch
    import torch.distributed as dist

    if args.actor_only:
        return actor_only(args, wd)
    if args.emulate_links:
        return central_emulated(args, wd)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.roctx:
        from apex_amd.utils import trace

        trace.enable(True)
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    if args.same_device:
        local_rank = 0
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    topo = select_topology(args.topology, world)
    if args.reserve and topo != "central":
        from apex_amd.engine.apex import reserve_actor_stream

        reserve_actor_stream(device)  # before the process group draws its pool streams
    if world > 1 or args.force_dp:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
    wd.kick()
    pre = run_preflight(args, topo, device, wd) if world > 1 else None
    args.transport, args.transport_fallback = resolve_transport(args.transport, pre)
    if args.transport_fallback and rank == 0:
        print(f"preflight: IPC experience links unavailable ({args.transport_fallback}); "
              f"using the {args.transport} transport", file=sys.stderr)
    if args.algo == "aql":
        if topo == "central":
            return aql_central(args, rank, world, device, wd, pre)
        return aql(args, rank, world, device)
    if topo == "central":
        return central(args, rank, world, device, wd, pre)

    from apex_amd.engine.apex import ApexEngine, EngineConfig
    from apex_amd.engine.learner import LearnerConfig
    from apex_amd.parallel.dp import FlatGradAllReduce

    if args.scaling == "strong" and args.batch % world:
        raise SystemExit(f"--scaling strong needs --batch divisible by {world}")
    rank_batch = args.batch // world if args.scaling == "strong" else args.batch
    lc = LearnerConfig(batch_size=rank_batch, forward=args.forward, dtype=args.dtype, seed=args.seed + rank,
                       tree_ride=bool(args.tree_ride), draw_in_conv1=bool(args.draw_in_conv1))
    cfg = EngineConfig(n_envs=args.envs, n_actions=args.actions, replay_capacity=args.capacity,
                       threshold_size=args.threshold, actor_steps_per_learner_step=args.actor_steps,
                       actor_offset=rank * args.envs, total_actors=world * args.envs,
                       use_graphs=not args.no_graphs, overlap=args.overlap, seed=args.seed + 7919 * rank,
                       actor_at=args.actor_at,
                       learner=lc)
    dp = world > 1 or args.force_dp
    allreduce = None
    if dp and args.comm == "rccl" and args.backend == "nccl":
        from apex_amd.parallel.rccl import RcclGradAllReduce

        try:
            allreduce = RcclGradAllReduce(device, force=args.force_dp)
        except RuntimeError as e:  # every rank fails alike (bootstrap/config): torch collectives instead
            print(f"rank {rank}: direct RCCL communicator unavailable ({e}); using torch.distributed", file=sys.stderr)
    if dp and allreduce is None:
        allreduce = FlatGradAllReduce(world, force=args.force_dp)
    sharded = dp and not args.local_sampling
    from apex_amd.parallel.rccl import RcclGradAllReduce as _Rccl

    cfg.dp_graph = bool(args.dp_graph and isinstance(allreduce, _Rccl))  # capture needs the direct communicator
    eng = ApexEngine(cfg, device, allreduce=allreduce, sharded=sharded, force_collectives=args.force_dp)
    if world > 1:  # identical initial weights on every replica (RCCL broadcast from rank 0)
        from apex_amd.parallel.broadcast import broadcast_flat

        broadcast_flat(eng.learner.flat, src=0)
        eng.learner.refresh_packed()
        eng.learner.sync_target()
        eng.learner.copy_params_to(eng.actor_flat)

    t_fill = time.perf_counter()
    eng.fill(args.capacity + 8 * args.envs if args.fill else args.threshold)
    torch.cuda.synchronize(device)
    t_fill = time.perf_counter() - t_fill
    wd.kick()
    if not args.no_graphs:
        eng.capture(warm_replays=args.graph_warm)
    wd.kick()
    for _ in range(args.warmup):
        eng.train_step()
    torch.cuda.synchronize(device)
    wd.kick()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.train_step()
    t_host = time.perf_counter() - t0  # host enqueue time (the GPU may still be running)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    host_launch = _host_launch_cost(eng, device)  # extra untimed steps after the timed region
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    wd.kick()
    for _ in range(args.profile_steps):
        eng.train_step()
    torch.cuda.synchronize(device)
    wd.off()

    rccl_ranks = allreduce.comm.count() if isinstance(allreduce, _Rccl) else None
    stats = eng.learner.stats()
    updates_per_s = args.steps / dt                # synchronous optimizer updates (all ranks step together)
    samples_per_s = world * rank_batch * args.steps / dt
    batches_per_s = samples_per_s / 512.0          # the reference's unit: batches of 512 per second
    frames_per_s = world * args.steps * args.actor_steps * eng.frames_per_actor_step / dt
    if rank == 0:
        out = {
            "metric": "learner SGD steps/sec + actor frames/sec, Ape-X DQN Atari at 1/2/4/8 MI355X",
            "value": round(batches_per_s, 3),
            "unit": ("learner batches of 512 sampled transitions per second, whole job (= SGD steps/s at N=1)"
                     if world == 1 else
                     f"sampled transitions/s / 512 of {world} data-parallel learners at global batch {512 * world} "
                     f"(sample throughput, NOT single-learner SGD steps/s: see optimizer_updates_per_s)"),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * dt / args.steps, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": round(batches_per_s / REFERENCE_BATCHES_PER_S, 2),
            "dtype": args.dtype,
            "data": "synthetic (GPU-rendered Atari-shaped 84x84x4 u8 frames, random-init weights)",
            "config": {
                "model": "Ape-X dueling double DQN, Nature-CNN trunk, 128-hidden dueling heads, 18 actions",
                "global_batch": rank_batch * world,
                "batch_per_rank": rank_batch,
                "seq_len": 3,
                "seq_len_meaning": "n-step return horizon (frame stack 4)",
                "parallelism": f"dp{world}" + ("-forced" if args.force_dp and world == 1 else ""),
                "dp_comm": (type(allreduce).__name__ if allreduce is not None else None),
                "replay_sampling": "global PER over shards (mass all-gather)" if sharded else "per-shard PER",
                "replay_capacity_per_gpu": args.capacity,
                "envs_per_gpu": args.envs,
                "actor_steps_per_learner_step": args.actor_steps,
                "optimizer": "centered RMSprop lr 6.25e-5 alpha .95 eps 1.5e-7, clip 40",
                "per": "alpha 0.6 beta 0.4, stratified proportional, fanout-64 HBM tree",
                "batch_pipeline": ("drawn inside the conv1 forward launch" if eng.learner.draws_in_conv1
                                   else "sampled at the step start") + ", 3-pass forward",
                "forward": args.forward,
                "fp32_gemms": "exact 3-term bf16 split (x6) on MFMA, fp32 accumulate" if args.dtype == "fp32" else None,
                "hip_graphs": not args.no_graphs,
                "graph_warm_replays": 0 if args.no_graphs else args.graph_warm,
                "actor_learner_overlap": args.overlap, "actor_at": args.actor_at,
                "tree_write": ("riders of the trunk backward's launches" if eng.learner.tree_rides_used
                               else "forked tree stream"),
                "dp_graph": eng._g_dp is not None,
                # ranks the communicators themselves report: RCCL's ncclCommCount on the direct
                # gradient communicator, else the torch.distributed group size
                "rccl_ranks": rccl_ranks,
                "process_group_ranks": dist.get_world_size() if dist.is_initialized() else 1,
                "process_group_backend": dist.get_backend() if dist.is_initialized() else None,
            },
            "optimizer_updates_per_s": round(updates_per_s, 3),
            "actor_frames_per_sec": round(frames_per_s, 1),
            "learner_samples_per_sec": round(samples_per_s, 1),
            "vs_paper_19_batches_per_s": round(batches_per_s / PAPER_BATCHES_PER_S, 2),
            "replay_fill_seconds": round(t_fill, 3),
            "replay_bytes_per_gpu": eng.replay.nbytes(),
            "replay_live_transitions": int((eng.replay.leaf_sum > 0).sum().item()),
            "replay_slots_written": int(eng.replay.filled.item()),
            # wall time of the enqueue loop: includes waiting on a full launch queue (back-pressure)
            "host_enqueue_ms_per_step": round(1000.0 * t_host / args.steps, 4),
            # one train_step's host cost with the GPU idle (no back-pressure), median of 20
            "host_launch_ms_per_step": round(1000.0 * host_launch, 4),
            "last_loss": round(stats["loss"], 6),
            "last_grad_norm_l2": round(stats["grad_norm_l2"], 6),
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def aql(args, rank, world, device):
    """GPU AQL engine (engine/aql.py), AQL_dis defaults: batch 32, propose 1 + uniform 50
    candidates, Adam lr 1e-3, n-step 1; replay ratio of the reference (one SGD step per 32
    new transitions).  ``value`` = learner SGD steps/s (whole job); actor env steps/s beside.
    Multi-GPU: independent engines per rank (no published AQL scaling number to compare)."""
    import torch
    import torch.distributed as dist

    from apex_amd.engine.aql import AQLEngine, AQLEngineConfig

    cap = min(args.capacity, 1_000_000)
    cfg = AQLEngineConfig(env_id=args.aql_env, n_envs=args.envs, capacity=cap, seed=args.seed + rank,
                          actor_offset=rank * args.envs, total_actors=world * args.envs, overlap=args.aql_overlap)
    eng = AQLEngine(cfg, device)
    t_fill = time.perf_counter()
    eng.fill(max(1024, 4 * args.envs))
    torch.cuda.synchronize(device)
    t_fill = time.perf_counter() - t_fill
    if not args.no_graphs:
        eng.capture()
    for _ in range(args.warmup):
        eng.iteration()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.iteration()
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    st = eng.learner.stats()
    eps = eng.finished_episodes()
    sgd = world * args.steps * eng.K / dt
    env_steps = world * args.steps * eng.E / dt
    if rank == 0:
        print(json.dumps({
            "metric": "AQL learner SGD steps/sec + actor env steps/sec (AQL_dis, BipedalWalker-shaped)",
            "value": round(sgd, 1), "unit": "learner SGD steps (batch 32) per second, whole job",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000.0 * dt / args.steps, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (GPU BipedalWalker-shaped env, random-init weights)",
            "config": {"model": f"AQL NoisyNet critic + proposal, {eng.obs}-d obs, {eng.adim}-d action, "
                                f"T={eng.T} candidates", "global_batch": cfg.batch_size * world, "seq_len": 1,
                       "parallelism": f"independent x{world}", "env": cfg.env_id, "envs_per_gpu": eng.E,
                       "sgd_steps_per_iteration": eng.K, "replay_capacity_per_gpu": cap,
                       "acting": ("own HIP stream beside the learner (staged transitions)" if eng.overlap
                                  else "serial before the learner steps"),
                       "learner_launches_per_step": 4 if eng.learner.fused else 7,
                       "optimizer": "Adam lr 1e-3 x2 (critic, proposal), clip 40 each"},
            "actor_env_steps_per_sec": round(env_steps, 1),
            "learner_samples_per_sec": round(sgd * cfg.batch_size, 1),
            "host_enqueue_ms_per_step": round(1000.0 * t_host / args.steps, 4),
            "replay_fill_seconds": round(t_fill, 3),
            "last_loss_q": round(st["loss_q"], 6), "last_loss_proposal": round(st["loss_proposal"], 6),
            "episodes_finished": len(eps),
            "mean_episode_return": round(float(np.mean([r for r, _ in eps])), 3) if eps else None,
        }), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def aql_central(args, rank, world, device, wd, pre=None):
    """Distributed AQL_dis (BASELINE config 4; the default for --algo aql with N>1): rank 0 =
    THE AQL learner (batch 32, AQL_dis.py:31-47) + the one replay, ranks 1.. = actor GPUs
    with ``--envs`` envs each pushing raw (s, a, r, s', d, a_mu) rows over HIP IPC
    (engine/central_aql.py; AQL_dis.py:50-53,109-126).  One rank-0 iteration = ingest (<= one
    packet per actor) + the SGD steps its rows pay for (at most K = (N-1) * envs / 32: the
    reference replay ratio, one step per 32 recorded transitions) + a weight publish.  ``value`` = learner SGD steps/s (the device step counter: the ingest's
    step gate runs only the steps the applied rows pay for); actor env steps/s = rows that
    reached the replay during the timed window."""
    import torch
    import torch.distributed as dist

    from apex_amd.engine.aql import AQLEngineConfig
    from apex_amd.engine.central_aql import CentralAQLEngine

    cap = min(args.capacity, 1_000_000)
    cfg = AQLEngineConfig(env_id=args.aql_env, n_envs=args.envs, capacity=cap, seed=args.seed)
    eng = CentralAQLEngine(cfg, device, rank, world, paced=not args.unpaced, transport=args.transport)
    wd.kick()
    if rank != 0:
        if not args.no_graphs:
            eng.capture()
        while eng.iteration():
            wd.kick(every=5.0)
        torch.cuda.synchronize(device)
        wd.off()
        dist.destroy_process_group()
        return
    t_fill = time.perf_counter()
    eng.fill()
    torch.cuda.synchronize(device)
    t_fill = time.perf_counter() - t_fill
    wd.kick()
    if not args.no_graphs:
        eng.capture()
    for _ in range(args.warmup):
        eng.iteration()
    torch.cuda.synchronize(device)
    wd.kick()
    a0 = sum(eng.applied.values())
    s0 = eng.sgd_steps()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.iteration()
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    packets = sum(eng.applied.values()) - a0
    n_sgd = eng.sgd_steps() - s0
    sgd = n_sgd / dt
    wd.kick()
    st = eng.eng.learner.stats()
    links = eng.close()
    wd.off()
    e = eng.eng
    print(json.dumps({
        "metric": "AQL learner SGD steps/sec + actor env steps/sec (AQL_dis, BipedalWalker-shaped)",
        "value": round(sgd, 1), "unit": "learner SGD steps (batch 32) per second, one central learner",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1000.0 * dt / args.steps, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (GPU BipedalWalker-shaped env, random-init weights)",
        "config": {"model": f"AQL NoisyNet critic + proposal, {e.obs}-d obs, {e.adim}-d action, T={e.T} candidates",
                   "global_batch": cfg.batch_size, "seq_len": 1, "parallelism": f"central1+actors{world - 1}",
                   "topology": "AQL learner + replay on rank 0, actor GPUs push rows over "
                               + ("HIP IPC" if eng.transport == "ipc" else "torch.distributed p2p links"),
                   "env": cfg.env_id, "envs_per_actor_gpu": args.envs, "sgd_steps_per_iteration": eng.K,
                   "replay_capacity": cap, "optimizer": "Adam lr 1e-3 x2 (critic, proposal), clip 40 each"},
        "actor_env_steps_per_sec": round(packets * eng.E / dt, 1),
        "packets_applied_per_iteration": round(packets / args.steps, 3),
        # the reference replay ratio is one SGD step per `batch` recorded transitions
        # (AQL_dis.py:117-118); the device step gate holds it whatever the actors' pace
        "sgd_steps_per_transition_x_batch": round(n_sgd * cfg.batch_size / max(1, packets * eng.E), 4),
        "learner_samples_per_sec": round(sgd * cfg.batch_size, 1),
        "replay_fill_seconds": round(t_fill, 3), "links": links,
        "links_complete": all(links["applied"][r] == links.get("sent", {}).get(r, links["applied"][r])
                              for r in links["live"]),
        "transport": eng.transport, "transport_fallback": getattr(args, "transport_fallback", None),
        "iterations": eng.iterations, "learner_spins": eng.spins, "target_syncs": len(e.target_syncs),
        "preflight": pre,
        "timing": "rank 0 (the one learner) between two device syncs; actor ranks act continuously",
        "last_loss_q": round(st["loss_q"], 6), "last_loss_proposal": round(st["loss_proposal"], 6),
    }), flush=True)
    dist.destroy_process_group()


# one actor GPU's unpaced frames/s by envs per GPU (bench.py --actor-only on MI355X,
# profiles/r6_central_capacity.md); interpolated log-linearly in E
ACTOR_GPU_CAPACITY_FPS = {256: 9.78e6, 512: 16.25e6, 1024: 22.0e6, 2048: 25.3e6}


def actor_gpu_capacity(E: int) -> float:
    pts = sorted(ACTOR_GPU_CAPACITY_FPS.items())
    if E <= pts[0][0]:
        return pts[0][1] * E / pts[0][0]
    for (e0, f0), (e1, f1) in zip(pts, pts[1:]):
        if E <= e1:
            w = (np.log(E) - np.log(e0)) / (np.log(e1) - np.log(e0))
            return float(f0 + w * (f1 - f0))
    return pts[-1][1]


def central_envs(args, n_links: int) -> int:
    """Envs per actor GPU of the central topology: --central-envs, or (auto) the row budget
    rank 0's learner absorbs at >= 95 % of the 1-GPU engine, split over the links."""
    if str(args.central_envs) != "auto":
        return int(args.central_envs)
    return min(2048, max(CENTRAL_MIN_ENVS, CENTRAL_ROW_BUDGET // max(1, n_links) // 64 * 64))


def central(args, rank, world, device, wd, pre=None, emulate: int = 0):
    """Central-replay topology (BASELINE config 3; the default for N>1), asynchronous:
    rank 0 = THE learner (batch 512, the reference's single learner, origin_repo/learner.py:
    134-175) + the one replay, ranks 1.. = actor GPUs pushing experience over their own
    HIP IPC links (credit window 3, conflated params; origin_repo/actor.py:105-115).
    ``value`` = learner SGD steps/s (one learner, batch 512: global work per step fixed ->
    "strong"); actor frames/s = frames that reached the replay during the timed window.
    Only rank 0 takes timed steps; the actor ranks act continuously until it stops them."""
    import torch
    import torch.distributed as dist

    from apex_amd.engine.apex import EngineConfig
    from apex_amd.engine.central import CentralApexEngine
    from apex_amd.engine.learner import LearnerConfig

    if world < 2:
        raise SystemExit("--topology central needs >= 2 ranks")
    lc = LearnerConfig(batch_size=args.batch, forward=args.forward, dtype=args.dtype, seed=args.seed,
                       tree_ride=bool(args.tree_ride), draw_in_conv1=bool(args.draw_in_conv1))
    E = central_envs(args, world - 1)
    cfg = EngineConfig(n_envs=E, n_actions=args.actions, replay_capacity=args.capacity,
                       threshold_size=args.threshold, actor_steps_per_learner_step=args.actor_steps,
                       use_graphs=not args.no_graphs, seed=args.seed, learner=lc)
    eng = CentralApexEngine(cfg, device, rank, world, paced=not args.unpaced, transport=args.transport,
                            emulate_links=emulate)
    wd.kick()
    if rank != 0:  # actor GPU: act and push until the learner stops this link
        if not args.no_graphs:
            eng.capture()
        while eng.train_step():
            wd.kick(every=5.0)
        torch.cuda.synchronize(device)
        wd.off()
        dist.destroy_process_group()
        return
    t_fill = time.perf_counter()
    eng.fill(timeout=300.0)
    torch.cuda.synchronize(device)
    t_fill = time.perf_counter() - t_fill
    wd.kick()
    if not args.no_graphs:
        eng.capture()
        for _ in range(args.graph_warm):  # real steps, back to back (see --graph-warm)
            eng.train_step()
    for _ in range(args.warmup):
        eng.train_step()
    torch.cuda.synchronize(device)
    wd.kick()
    a0 = sum(eng.applied.values())
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.train_step()
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    packets = sum(eng.applied.values()) - a0
    wd.kick()
    links = eng.close()
    wd.off()
    st = eng.learner.stats()
    steps_per_s = args.steps / dt
    print(json.dumps({
        "metric": "learner SGD steps/sec + actor frames/sec, Ape-X DQN Atari at 1/2/4/8 MI355X",
        "value": round(steps_per_s, 3), "unit": "learner SGD steps/s (one central learner, batch 512)",
        "n_gpus": 1 if emulate else world, "steps": args.steps, "warmup": args.warmup,
        "graph_warm_replays": 0 if args.no_graphs else args.graph_warm,
        "ms_per_step": round(1000.0 * dt / args.steps, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": round(steps_per_s / REFERENCE_BATCHES_PER_S, 2), "dtype": args.dtype,
        "data": "synthetic (GPU-rendered Atari-shaped 84x84x4 u8 frames, random-init weights)",
        "config": {"model": "Ape-X dueling double DQN, Nature-CNN trunk, 128-hidden dueling heads, 18 actions",
                   "global_batch": args.batch, "seq_len": 3,
                   "parallelism": (f"central1+emulated_links{emulate}" if emulate else f"central1+actors{world - 1}"),
                   "topology": "central replay on rank 0, async experience links over "
                               + ("HIP IPC (xGMI peer copies)" if eng.transport == "ipc" else args.backend),
                   "actor_pacing": "free" if args.unpaced else f"{args.actor_steps} packet/learner step/actor",
                   "replay_capacity": eng.C_r * (world - 1), "envs_per_actor_gpu": E},
        "actor_frames_per_sec": round(packets * eng.frames_per_actor_step / dt, 1),
        "packets_applied_per_learner_step": round(packets / args.steps, 3),
        # sampled transitions per new transition that reached the replay in the window
        "replay_ratio": round(args.steps * args.batch / max(1, packets * E), 4),
        # each actor GPU's frames/s against what one actor GPU generates unpaced at this E
        # (bench.py --actor-only on MI355X, ACTOR_GPU_CAPACITY_FPS)
        "actor_gpu_utilisation": round(packets * eng.frames_per_actor_step / dt / (world - 1)
                                       / actor_gpu_capacity(E), 3),
        "replay_fill_seconds": round(t_fill, 3), "links": links,
        "links_complete": all(links["applied"][r] == links.get("sent", {}).get(r, links["applied"][r]) for r in links["live"]),
        "transport": eng.transport, "transport_fallback": getattr(args, "transport_fallback", None),
        "preflight": pre,
        "timing": "rank 0 (the one learner) between two device syncs; actor ranks act continuously",
        "last_loss": round(st["loss"], 6), "last_grad_norm_l2": round(st["grad_norm_l2"], 6),
    }), flush=True)
    dist.destroy_process_group()




def central_emulated(args, wd):
    """``--emulate-links R``: BASELINE config 3's rank 0 on one GPU -- the central learner
    with R actor links emulated in-process (parallel.ipc.EmulatedActorLinks: one synthetic
    packet per link per learner step, credit permitting, written into the real IPC ring and
    applied by the real in-graph ingest + batched tree write).  Not a scaling number: the
    learner's steps/s under the ingest load of N = R + 1 GPUs (is rank 0 still
    at the 1-GPU rate with 7 links?)."""
    import torch
    import torch.distributed as dist

    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
        raise SystemExit("--emulate-links runs in ONE process")
    torch.cuda.set_device(0)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29000 + os.getpid() % 1000))
    dist.init_process_group("gloo", rank=0, world_size=1)  # (the store the IPC handshake keys live in)
    return central(args, 0, args.emulate_links + 1, torch.device("cuda", 0), wd, None, emulate=args.emulate_links)


def actor_only(args, wd):
    """``--actor-only E,..``: what one actor GPU of the central topology generates unpaced --
    per actor step: batched inference of its E envs (eps-greedy in the heads kernel), the env
    step, the n-step rows + priorities into its local mirror, the packet staging launch and a
    device copy of the packet (standing in for the xGMI push) -- graph-captured and timed
    back to back.  Frames/s = 4 emulator frames per env step (action repeat 4)."""
    import torch

    from apex_amd import ops
    from apex_amd.engine.apex import EngineConfig
    from apex_amd.engine.central import actor_rank_step, build_actor_rank, region_geometry
    from apex_amd.engine.learner import LearnerConfig
    from apex_amd.parallel.ipc import packet_bytes

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    hip = ops.hip()
    rows = []
    for E in [int(x) for x in args.actor_only.split(",") if x]:
        cfg = EngineConfig(n_envs=E, n_actions=args.actions, replay_capacity=args.capacity, seed=args.seed,
                           learner=LearnerConfig(batch_size=args.batch, forward="hip", dtype=args.dtype))
        R = 7  # the actor ranks of one 8-GPU node: each rank's region of the central replay
        C_r, F_r = region_geometry(cfg, R)
        a = build_actor_rank(cfg, dev, 1, R, C_r, F_r)
        pkt = torch.empty(packet_bytes(E), dtype=torch.uint8, device=dev)
        dst = torch.empty_like(pkt)

        def step():
            actor_rank_step(hip, a, pkt)
            dst.copy_(pkt)

        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(3):
                step()
        torch.cuda.current_stream(dev).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        for _ in range(args.warmup):
            g.replay()
        torch.cuda.synchronize(dev)
        wd.kick()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            g.replay()
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        wd.kick()
        rows.append({"envs": E, "actor_steps_per_sec": round(args.steps / dt, 1),
                     "frames_per_sec": round(args.steps * E * 4 / dt, 1),
                     "us_per_actor_step": round(1e6 * dt / args.steps, 2),
                     "packet_bytes": packet_bytes(E)})
        del a, g
        torch.cuda.empty_cache()
    wd.off()
    best = max(rows, key=lambda r: r["frames_per_sec"])
    print(json.dumps({
        "metric": "actor frames/sec of one central-topology actor GPU (unpaced)",
        "value": best["frames_per_sec"], "unit": "emulator frames/s (4 per env step) of one actor rank",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "higher_is_better": True, "vs_baseline": None,
        "dtype": args.dtype, "data": "synthetic (GPU-rendered Atari-shaped 84x84x4 u8 frames, random-init weights)",
        "config": {"model": "Ape-X dueling double DQN actor (Nature-CNN, 18 actions)", "parallelism": "actor rank",
                   "work_per_step": "inference + eps-greedy, env step, n-step rows + priorities, packet staging, "
                                    "packet copy"},
        "per_envs": rows,
    }), flush=True)


if __name__ == "__main__":
    main()
