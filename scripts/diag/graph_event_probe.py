#!/usr/bin/env python
"""Probe: an EXTERNAL event recorded inside a captured hipGraph (torch.cuda.Event(external=True):
an event-record node) and waited on by another stream between graph launches -- the pattern a
learner graph needs to hand its mid-step point to a second graph (the priority-tree work) without
a fork/join inside the learner graph.  Checks ordering on the device and times the hand-off.

graph A on stream L: k1 (sleep) -> x = 1 -> record ev_mid (external) -> k2 (sleep) -> x = 2
stream T, per replay: wait ev_mid -> graph B: y = x (must read 1 or 2, never 0) -> record ev_b
L waits ev_b before the next replay of A.
"""
import sys
import time

import torch


def main():
    dev = torch.device("cuda", 0)
    L = torch.cuda.Stream(device=dev)
    T = torch.cuda.Stream(device=dev)
    x = torch.zeros(1, device=dev)
    y = torch.zeros(64, device=dev)
    ev_mid = torch.cuda.Event(external=True)
    ev_b = torch.cuda.Event()
    ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.stream(L):
        with torch.cuda.graph(ga, stream=L):
            torch.cuda._sleep(200_000)
            x.fill_(1.0)
            ev_mid.record(L)
            torch.cuda._sleep(400_000)
            x.fill_(2.0)
    k = torch.zeros(1, dtype=torch.long, device=dev)
    with torch.cuda.stream(T):
        with torch.cuda.graph(gb, stream=T):
            y.copy_(x.expand(64))
    torch.cuda.synchronize()
    bad, mid = 0, 0
    for i in range(200):
        with torch.cuda.stream(L):
            x.zero_()
            ga.replay()
        T.wait_event(ev_mid)
        with torch.cuda.stream(T):
            gb.replay()
            ev_b.record(T)
        L.wait_event(ev_b)
        torch.cuda.synchronize()
        v = float(y[0])
        if v not in (1.0, 2.0):
            bad += 1
        mid += v == 1.0
    # mid: B ran between the two fills (the event fired mid-graph, not at the graph's end)
    print(f"ordering: {200 - bad}/200 replays read x after the mid-graph event (bad={bad}); "
          f"{mid}/200 read it mid-graph")
    # timing: A alone vs A with the hand-off to B each replay
    for mode in ("alone", "handoff"):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(200):
            with torch.cuda.stream(L):
                ga.replay()
            if mode == "handoff":
                T.wait_event(ev_mid)
                with torch.cuda.stream(T):
                    gb.replay()
                    ev_b.record(T)
                L.wait_event(ev_b)
        torch.cuda.synchronize()
        print(f"{mode}: {1e6 * (time.perf_counter() - t0) / 200:.1f} us per replay")
    return 0 if bad == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
