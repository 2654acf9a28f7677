"""HIP IPC primitives of the central transport (parallel/ipc.py, ops/csrc/ipc.cpp) between
two processes on ONE MI355X: an uncached arena exported with hipIpcGetMemHandle, a peer
process writing into it with hipMemcpyAsync + a system-scope sequence store, the owner's
kernels storing into a hipHostRegister'ed /dev/shm control block that the other process
reads with plain CPU loads."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _body(rank, port, q):
    import time
    import traceback
    from datetime import timedelta

    try:
        import torch.distributed as dist

        from apex_amd import ops
        from apex_amd.parallel.ipc import ControlBlock

        torch.cuda.set_device(0)
        store = dist.TCPStore("127.0.0.1", port, 2, rank == 0, timedelta(seconds=60))
        h = ops.hip()
        N = 1 << 20
        s = torch.cuda.current_stream().cuda_stream
        if rank == 0:
            arena = h.ipc_alloc(N + 4096, 2)
            ctrl = ControlBlock(f"apex_ipc_test_{os.getpid()}", 2, create=True)
            dev = ctrl.register(h)
            store.set("handle", h.ipc_handle(arena))
            store.set("shm", ctrl.name)
            host = torch.zeros(N // 4 + 2, dtype=torch.int32)
            seen = None
            deadline = time.monotonic() + 60
            while time.monotonic() < deadline:  # poll the sequence word the peer stores after its copy
                h.memcpy_sync(host.data_ptr() + N, arena + N, 8)
                if int(host[N // 4]) == 7:
                    seen = True
                    break
                time.sleep(0.001)
            h.memcpy_sync(host.data_ptr(), arena, N)
            ok = bool(seen) and torch.equal(host[:N // 4], torch.arange(N // 4, dtype=torch.int32) * 3)
            h.ipc_flag(dev + 8 * ctrl.off("consumed"), 1234, s)  # kernel store into shm
            torch.cuda.synchronize()
            store.wait(["done"], timedelta(seconds=60))
            ctrl.unlink()
            ctrl.close()
            h.ipc_free(arena)
            q.put((0, ok))
        else:
            store.wait(["handle", "shm"], timedelta(seconds=60))
            remote = h.ipc_open(store.get("handle"), 0)
            ctrl = ControlBlock(store.get("shm").decode(), 2, create=False)
            src = (torch.arange(N // 4, dtype=torch.int32, device="cuda") * 3)
            h.memcpy_async(remote, src.data_ptr(), N, s)
            h.ipc_flag(remote + N, 7, s)
            torch.cuda.synchronize()
            deadline = time.monotonic() + 60
            got = None
            while time.monotonic() < deadline:
                v = int(ctrl.view("consumed")[0])
                if v == 1234:
                    got = v
                    break
                time.sleep(0.001)
            store.set("done", "1")
            h.ipc_close(remote)
            q.put((1, got == 1234))
    except Exception:
        q.put((rank, "ERROR " + traceback.format_exc()))
    q.close()
    q.join_thread()
    os._exit(0)


def test_ipc_arena_peer_copy_and_shm_control(cuda):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_body, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(2):
        r, res = q.get(timeout=150)
        out[r] = res
    for p in procs:
        p.join(30)
        if p.is_alive():
            p.kill()
    assert out[0] is True, out[0]   # the peer's bytes landed before its sequence word
    assert out[1] is True, out[1]   # the owner's kernel store reached the other process's CPU


def _params_body(rank, port, q, seconds, delay_cycles):
    import time
    import traceback
    from datetime import timedelta

    try:
        import torch.distributed as dist

        from apex_amd.engine.aql import AQLReplay
        from apex_amd.parallel.experience import STOP
        from apex_amd.parallel.ipc import IpcActorLink, IpcLearnerLinks, aql_packet_floats

        torch.cuda.set_device(0)
        store = dist.TCPStore("127.0.0.1", port, 2, rank == 0, timedelta(seconds=60))
        E, P, obs, T, adim = 8, 1 << 20, 4, 3, 1
        flat = torch.zeros(P, dtype=torch.float32, device="cuda")
        if rank == 0:  # the writer: a new parameter version every "iteration", no clock floor
            rp = AQLReplay(1024, obs, T, adim, device="cuda")
            links = IpcLearnerLinks.for_aql(1, 3, E, P, rp, store, "pt", "cuda", log=None)
            store.set("ready", "1")
            n, t_end = 0, time.monotonic() + seconds
            while time.monotonic() < t_end:
                flat.fill_(float(n))
                links.publish(flat)
                torch.cuda._sleep(20000)  # ~10 us of "learner iteration"
                n += 1
                if n % 64 == 0:
                    torch.cuda.synchronize()
            st = links.close(timeout=60)
            q.put((0, {"published": n, "version": st["params_version"]}))
        else:  # the reader: every pull queued behind ~ms of other work on its stream
            store.wait(["ready"], timedelta(seconds=60))
            pkt = torch.zeros(aql_packet_floats(E, obs, T * adim), dtype=torch.float32, device="cuda")
            link = IpcActorLink(1, store, "pt", flat, pkt, "cuda")
            polls, installs, torn, last = 0, 0, 0, 0
            while True:
                torch.cuda._sleep(delay_cycles)  # queued work ahead of the parameter copy
                v = link.poll_params()
                polls += 1
                if v == STOP:
                    break
                if v is None:
                    continue
                lo, hi = float(flat.min()), float(flat.max())
                torn += int(lo != hi)
                assert v > last
                last, installs = v, installs + 1
            q.put((1, {"polls": polls, "installs": installs, "torn": torn, "retried": link.pulls_retried}))
    except Exception:
        q.put((rank, "ERROR " + traceback.format_exc()))
    q.close()
    q.join_thread()
    os._exit(0)


def test_ipc_params_delayed_reader_installs_while_writer_publishes_every_iteration(cuda):
    """with the pinned K-buffer protocol (parallel/ipc.py) a reader whose
    copies sit behind ~2 ms of queued work still installs a clean (untorn) version on
    practically every poll while rank 0 publishes a new version every ~10 us -- no publish
    floor, no starvation."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_params_body, args=(r, port, q, 3.0, 4_000_000)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(2):
        r, res = q.get(timeout=150)
        out[r] = res
    for p in procs:
        p.join(30)
        if p.is_alive():
            p.kill()
    for r, res in out.items():
        assert not (isinstance(res, str) and res.startswith("ERROR")), f"rank {r}: {res}"
    w, rd = out[0], out[1]
    print(w, rd)
    assert w["published"] > 10 * rd["installs"]       # the writer ran far ahead of the reader
    assert rd["torn"] == 0 and rd["installs"] >= 20
    assert rd["retried"] <= 2 and rd["installs"] >= rd["polls"] - 3  # bounded polls per install
