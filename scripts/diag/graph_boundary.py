#!/usr/bin/env python
"""Where the fp32 DQN step's time goes beyond its learner kernels (timing only):

  (a) the overlapped engine's train_step (actor graph || learner graph, event waits);
  (b) the learner graphs alone, replayed back to back on one stream (no actor, no waits);
  (c) ONE graph holding two learner steps (both staging halves) -- (b) minus (c)/2 is the
      cost of a graph launch boundary;
  (d) / (e) / (f) the engine's event pattern with the whole actor graph / only its forward
      (+ eps-greedy heads) / only its env step + n-step staging beside the learner graph.

Each timed over ``--steps`` steps, round-robin ``--rounds`` times (MI355X, bench config)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    from apex_amd.engine.apex import ApexEngine, EngineConfig
    from apex_amd.engine.learner import LearnerConfig

    lc = LearnerConfig(batch_size=512, forward="hip", dtype="fp32")
    eng = ApexEngine(EngineConfig(learner=lc, threshold_size=50_000, overlap=True, use_graphs=True), "cuda:0")
    eng.fill(50_000)
    eng.capture(warm_replays=50)
    torch.cuda.synchronize()
    ga = eng._g_learn_a
    two = torch.cuda.CUDAGraph()
    with torch.cuda.graph(two, pool=eng._pool, capture_error_mode="thread_local"):
        for h in (0, 1):
            eng._learn_a(1 - h)
            eng._learn_b()
    torch.cuda.synchronize()
    apool = torch.cuda.graph_pool_handle()

    def actor_graphs(fn):
        return [eng._graph(lambda h=h: fn(h), apool) for h in (0, 1)]

    g_fwd = actor_graphs(lambda h: eng.actor_net(eng.replay.frames, eng.actor_ws, eng.actor.st["hist"],
                                                 act=eng.actor.act_args()))
    g_env = actor_graphs(lambda h: eng.actor.act_and_step(None, h, selected=True))
    torch.cuda.synchronize()
    # (g) timing probe only: the learner graphs WITHOUT the forked priority-tree branch (no tree
    # writes at all -- wrong replay semantics, kept out of every other case): its fork/join cost
    L = eng.learner
    fork, join = L._fork_point, L._tree_fork_end
    L._fork_point, L._tree_fork_end = (lambda: None), (lambda: None)
    g_notree = [eng._graph(lambda h=h: (eng._learn_a(1 - h), eng._learn_b()), eng._pool) for h in (0, 1)]

    # (h) timing probe only: the tree branch forked at the graph's start (it would write the
    # PREVIOUS step's priorities; here it races the sampling -- timing only) and joined after
    # the optimizer, i.e. no fork / join in the middle of the learner chain
    def root_fork(h):
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        L._tree_fork_begin(ev)
        eng._learn_a(1 - h)
        eng._learn_b()
        torch.cuda.current_stream().wait_stream(L.tree_stream)

    g_rootfork = [eng._graph(lambda h=h: root_fork(h), eng._pool) for h in (0, 1)]
    L._fork_point, L._tree_fork_end = fork, join
    torch.cuda.synchronize()
    eng._ev_learn.record(torch.cuda.current_stream())

    def step_with(gA, n):  # _train_step_overlap's event pattern (no publish / target sync)
        L, A = torch.cuda.current_stream(), eng._astream
        for _ in range(n):
            h = eng._half
            A.wait_event(eng._ev_learn)
            with torch.cuda.stream(A):
                gA[h].replay()
            eng._ev_actor[h].record(A)
            L.wait_event(eng._ev_actor[1 - h])
            ga[h].replay()
            eng._ev_learn.record(L)
            eng._half ^= 1

    def timed(fn, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        fn(n)
        e1.record()
        torch.cuda.synchronize()
        return 1000.0 * e0.elapsed_time(e1) / n

    def engine(n):
        for _ in range(n):
            eng.train_step()

    def learner_only(n):
        for i in range(n):
            ga[i & 1].replay()

    def two_step(n):
        for _ in range(n // 2):
            two.replay()

    cases = {"(a) train_step (actor || learner)": engine, "(b) learner graphs alone": learner_only,
             "(c) two learner steps per graph": two_step,
             "(d) learner || whole actor graph": lambda n: step_with(eng._g_actor, n),
             "(e) learner || actor forward only": lambda n: step_with(g_fwd, n),
             "(f) learner || actor env step + staging only": lambda n: step_with(g_env, n),
             "(g) learner graphs alone, no tree branch (probe)": lambda n: [g_notree[i & 1].replay() for i in range(n)],
             "(h) learner graphs alone, tree branch forked at the start (probe)":
                 lambda n: [g_rootfork[i & 1].replay() for i in range(n)]}
    res = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, fn in cases.items():
            fn(50)  # back at load before each timed case
            res[k].append(timed(fn, a.steps))
    for k, v in res.items():
        print(f"{k}: {sorted(v)[len(v) // 2]:.1f} us/step  {['%.1f' % x for x in v]}")


if __name__ == "__main__":
    main()
