"""bench.py's CPU-side contract: topology selection per N (BASELINE config 3 = the central
single-learner topology for every N > 1; the single-GPU engine at N = 1) and the
no-progress watchdog."""
import importlib.util
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("topology,world,want", [
    ("auto", 1, "single"), ("auto", 2, "central"), ("auto", 4, "central"), ("auto", 8, "central"),
    ("sharded", 1, "single"), ("sharded", 8, "sharded"), ("central", 3, "central")])
def test_topology_per_world(topology, world, want):
    assert _bench().select_topology(topology, world) == want


def test_central_needs_two_ranks():
    with pytest.raises(SystemExit):
        _bench().select_topology("central", 1)


def test_default_topology_is_auto():
    import argparse

    b = _bench()
    old = sys.argv
    sys.argv = ["bench.py"]
    try:
        a = b.parse()
    finally:
        sys.argv = old
    assert isinstance(a, argparse.Namespace)
    assert a.topology == "auto" and a.preflight and 0 < a.watchdog < 600 and a.launch_timeout < 600


def test_watchdog_fires_on_no_progress_and_not_while_kicked():
    code = ("import importlib.util,sys,time;"
            f"s=importlib.util.spec_from_file_location('b',{os.path.join(ROOT, 'bench.py')!r});"
            "b=importlib.util.module_from_spec(s);s.loader.exec_module(b);"
            "w=b.Watchdog(1.0);"
            "[ (time.sleep(0.3), w.kick()) for _ in range(6) ];"  # 1.8 s alive while kicked
            "print('survived',flush=True);time.sleep(3);print('not reached')")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert "survived" in p.stdout and "not reached" not in p.stdout
    assert p.returncode == 1 and "Timeout" in p.stderr  # faulthandler's stack dump


@pytest.mark.parametrize("links,want", [(1, 2048), (2, 1984), (3, 1344), (7, 640)])
def test_central_envs_split_the_row_budget(links, want):
    """Central topology: by default each actor GPU gets its share of rank 0's ingest budget
    (CENTRAL_ROW_BUDGET rows per learner step, multiples of 64 in 256..2048), so the frames that
    reach the replay grow with N while the learner holds its rate (a floor of CENTRAL_MIN_ENVS per
    actor GPU lets N = 8 deliver more than N = 4); an explicit value stands."""
    import types

    b = _bench()
    assert b.central_envs(types.SimpleNamespace(central_envs="auto"), links) == want
    assert links * want <= b.CENTRAL_ROW_BUDGET or want == b.CENTRAL_MIN_ENVS
    assert b.central_envs(types.SimpleNamespace(central_envs="320"), links) == 320


def test_actor_capacity_interpolates_measured_points():
    b = _bench()
    for e, fps in b.ACTOR_GPU_CAPACITY_FPS.items():
        assert b.actor_gpu_capacity(e) == pytest.approx(fps)
    assert b.ACTOR_GPU_CAPACITY_FPS[256] < b.actor_gpu_capacity(384) < b.ACTOR_GPU_CAPACITY_FPS[512]
