"""``bench.py --gpus N`` self-launch (parallel/spawn.py): N fresh rank processes with the
torchrun env, rank 0's output forwarded, the first failure stops every other rank."""
import json
import os
import subprocess
import sys
import time

import pytest

from apex_amd.parallel.spawn import run_ranks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys, time
r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
open(os.path.join(sys.argv[1], f"pid{r}"), "w").write(str(os.getpid()))
mode = sys.argv[2]
if mode == "ok":
    if r == 0:
        print(json.dumps({"rank": r, "world": w, "local": int(os.environ["LOCAL_RANK"]),
                          "addr": os.environ["MASTER_ADDR"], "port": int(os.environ["MASTER_PORT"])}), flush=True)
    sys.exit(0)
if mode == "fail1":
    if r == 1:
        time.sleep(0.5)
        sys.exit(3)
    time.sleep(120)
if mode == "hang":
    time.sleep(120)
"""


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    # a zombie still answers kill(0); treat it as gone
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split()[2] != "Z"
    except FileNotFoundError:
        return False


def _pids(d, n):
    return [int(open(os.path.join(d, f"pid{r}")).read()) for r in range(n) if os.path.exists(os.path.join(d, f"pid{r}"))]


def test_all_ranks_ok(tmp_path, capfd):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    assert run_ranks([sys.executable, str(script), str(tmp_path), "ok"], 4, timeout=60) == 0
    out = capfd.readouterr().out.strip().splitlines()
    rec = json.loads(out[-1])
    assert rec["world"] == 4 and rec["rank"] == 0 and rec["local"] == 0 and rec["addr"] == "127.0.0.1"
    assert len(_pids(tmp_path, 4)) == 4


def test_child_failure_stops_the_others(tmp_path):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    t0 = time.monotonic()
    code = run_ranks([sys.executable, str(script), str(tmp_path), "fail1"], 3, timeout=60, grace=2.0)
    assert code == 3
    assert time.monotonic() - t0 < 30
    pids = _pids(tmp_path, 3)
    assert len(pids) == 3 and not any(_alive(p) for p in pids)


def test_timeout_kills_every_rank(tmp_path):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    code = run_ranks([sys.executable, str(script), str(tmp_path), "hang"], 2, timeout=2.0, grace=2.0)
    assert code == 124
    assert not any(_alive(p) for p in _pids(tmp_path, 2))


def test_bench_self_launch_propagates_failure():
    """bench.py --gpus 2 without WORLD_SIZE launches 2 ranks itself; on this GPU-less
    host both ranks fail (no device) and the launcher exits non-zero, leaving nothing running."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""  # never reach a GPU even if this host had one
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--launch-timeout", "120"], env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode != 0
    assert "spawn: rank" in p.stderr
