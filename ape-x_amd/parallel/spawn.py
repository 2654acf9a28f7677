"""One-process-per-GPU launcher used when a script is started without
``torch.distributed.run`` (``bench.py --gpus N`` with no ``WORLD_SIZE`` in the env).

The parent never touches the GPU (no ``torch.cuda`` call, not even an import of
torch): it only picks a free rendezvous port on 127.0.0.1 and starts N fresh children
with ``subprocess.Popen`` (never ``exec``), each with ``RANK``, ``LOCAL_RANK``,
``WORLD_SIZE``, ``MASTER_ADDR`` and ``MASTER_PORT`` set, as torchrun would.  Children
share the parent's stdout/stderr, so rank 0's one JSON line reaches the caller as is.

Failure policy (the reference has none): the first child that exits
non-zero, or the wall-clock limit, ends the job -- every other child gets SIGTERM,
then SIGKILL after a grace period, and the parent exits with the failing child's code
(124 on timeout).  A SIGTERM/SIGINT to the parent is forwarded the same way, so no
rank outlives its launcher.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def rank_env(rank: int, world: int, port: int, base: dict | None = None, local_rank: int | None = None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank if local_rank is None else local_rank),
               WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world), GROUP_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return env


def _stop(procs: list[subprocess.Popen], grace: float = 10.0) -> None:
    for p in procs:
        if p.poll() is None:
            try:
                p.terminate()
            except OSError:
                pass
    deadline = time.monotonic() + grace
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def run_ranks(cmd: list[str], world: int, timeout: float = 3600.0, poll: float = 0.2,
              env: dict | None = None, grace: float = 10.0) -> int:
    """Run ``cmd`` as ``world`` ranks; returns 0 iff every rank exits 0 in time."""
    port = free_port()
    procs = [subprocess.Popen(cmd, env=rank_env(r, world, port, env)) for r in range(world)]
    fired = []

    def _forward(signum, _frame):
        fired.append(signum)

    old = {s: signal.signal(s, _forward) for s in (signal.SIGTERM, signal.SIGINT)}
    code = 0
    try:
        t0 = time.monotonic()
        while True:
            if fired:
                code = 128 + fired[0]
                print(f"spawn: signal {fired[0]}, stopping {world} ranks", file=sys.stderr, flush=True)
                break
            rcs = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(rcs) if c not in (None, 0)]
            if bad:
                r, code = bad[0]
                code = 128 - code if code < 0 else code  # killed by a signal: shell convention
                print(f"spawn: rank {r} exited with {code}, stopping the others", file=sys.stderr, flush=True)
                break
            if all(c == 0 for c in rcs):
                return 0
            if time.monotonic() - t0 > timeout:
                code = 124
                print(f"spawn: {timeout:.0f} s limit reached, stopping {world} ranks", file=sys.stderr, flush=True)
                break
            time.sleep(poll)
    finally:
        _stop(procs, grace)
        for s, h in old.items():
            # a handler installed outside Python (e.g. a profiler's preloaded library) reads
            # back as None and cannot be re-installed from here: leave ours in place then
            if h is not None:
                signal.signal(s, h)
    return code if code != 0 else 1
