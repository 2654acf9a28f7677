"""Single-host launcher for the role topology (the reference's run.sh / tmux deploy
scripts, origin_repo/run.sh:2-5, deploy/*.sh).

``python -m apex_amd.roles.launch --n-actors 4 [--no-eval] [--port P] -- [arguments.py flags]``

Starts replay (first: it hosts the rendezvous store), learner, evaluator and the
actors as child processes with the reference env vars (``ACTOR_ID``, ``N_ACTORS``,
``REPLAY_IP``, ``LEARNER_IP``), waits for the learner, then for the others (bounded),
and returns the learner's exit code.  Multi-host: run the same module commands on
each host with ``REPLAY_IP`` pointing at the replay host.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def role_cmd(role: str, flags: list[str]) -> list[str]:
    return [sys.executable, "-m", f"apex_amd.roles.{role}", *flags]


def launch(n_actors: int, flags: list[str], n_eval: int = 1, port: int = 29555, ip: str = "127.0.0.1",
           learner_flags=(), actor_flags=(), eval_flags=(), env_extra: dict | None = None, log_dir: str | None = None,
           timeout: float = 3600.0) -> dict:
    base = dict(os.environ)
    base.update({"N_ACTORS": str(n_actors), "N_EVAL": str(n_eval), "REPLAY_IP": ip, "LEARNER_IP": ip,
                 "APEX_PORT": str(port), "OMP_NUM_THREADS": "1"})
    base["PYTHONPATH"] = ROOT + os.pathsep + base.get("PYTHONPATH", "")
    base.update(env_extra or {})
    procs = {}

    def start(name, role, extra, env):
        out = open(os.path.join(log_dir, f"{name}.log"), "w") if log_dir else None
        procs[name] = (subprocess.Popen(role_cmd(role, [*flags, *extra]), env=env, cwd=ROOT, stdout=out,
                                        stderr=subprocess.STDOUT if out else None), out)

    if log_dir:
        os.makedirs(log_dir, exist_ok=True)
    start("replay", "replay", [], base)
    time.sleep(0.5)
    start("learner", "learner", list(learner_flags), base)
    if n_eval:
        start("eval", "evaluator", list(eval_flags), base)
    for i in range(n_actors):
        start(f"actor{i}", "actor", list(actor_flags), {**base, "ACTOR_ID": str(i)})
    codes = {}
    try:
        learner = procs["learner"][0]
        learner.wait(timeout=timeout)
        deadline = time.time() + 120.0
        for name, (p, _) in procs.items():
            try:
                p.wait(timeout=max(1.0, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    finally:
        for name, (p, out) in procs.items():
            if p.poll() is None:
                p.kill()
                p.wait()
            codes[name] = p.returncode
            if out:
                out.close()
    return codes


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if "--" in argv:
        i = argv.index("--")
        own, flags = argv[:i], argv[i + 1:]
    else:
        own, flags = argv, []
    p = argparse.ArgumentParser(description="launch replay + learner + evaluator + N actors on this host")
    p.add_argument("--n-actors", type=int, default=int(os.environ.get("N_ACTORS", 1)))
    p.add_argument("--no-eval", action="store_true")
    p.add_argument("--port", type=int, default=29555)
    p.add_argument("--log-dir", default=None)
    a = p.parse_args(own)
    codes = launch(a.n_actors, flags, n_eval=0 if a.no_eval else 1, port=a.port, log_dir=a.log_dir)
    print(codes)
    sys.exit(codes.get("learner", 1))


if __name__ == "__main__":
    main()
