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
