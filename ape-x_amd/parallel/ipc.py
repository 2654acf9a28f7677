"""Central-replay experience transport over HIP IPC (SURVEY §2.4 M1/M4, §5.3, §5.8;
reference actor.py:40-49,105-115, replay.py:77-146, learner.py:57-68).

MI355X-native replacement of the reference's ZeroMQ actor -> replay pushes and PUB/SUB
parameter publish, for actor GPUs on the same node (xGMI):

* **Data plane (device memory, no host on the path).**  Rank 0 allocates one *uncached*
  arena in its HBM (``ipc_alloc(mode=2)``: loads and stores bypass L2, so bytes that peers
  write over xGMI are never hidden behind a stale L2 line) holding, per actor link r, a
  ring of ``D`` packet slots and their sequence words, plus a double-buffered parameter
  block.  The arena is exported once with ``hipIpcGetMemHandle`` through the TCPStore.
  An actor pushes a packet (one actor step: E new frames + E transition rows) with ONE
  ``hipMemcpyAsync`` into its next ring slot over xGMI and then, stream-ordered behind the
  copy, a one-thread system-scope release store of the packet number into the slot's
  sequence word.  Rank 0 ingests inside its learner hipGraph (``ipc_ingest``: scan the
  sequence words with system-scope acquires, scatter every ready packet into the link's
  replay region, release the slots), followed by one masked tree write -- no Python
  polling, no receive left posted, no host sync per step.
* **Control plane (host memory).**  A small ``/dev/shm`` control block, mapped into every
  process (rank 0 also registers it with ``hipHostRegister`` so its kernels can store
  into it): per-link *consumed* counters written by rank 0's release kernel (the actors'
  credit window, actor.py:105-115: at most ``D`` packets in flight), the published
  parameter version, per-link heartbeat counters, drop flags, the stop flag and stop
  acknowledgements.  The actors read and write it with plain CPU loads / stores.
* **Parameters** (conflated, learner.py:57-68 PUB/SUB CONFLATE=1): ``K = R + 2`` parameter
  buffers.  The published word in the control block is ``v << 8 | b``: version ``v`` lives in
  buffer ``b``.  A reader *pins* the word it is about to pull (its pin slot), pulls buffer ``b``
  with one peer copy, then checks that buffer's *begin* word still reads ``v`` (nobody began
  rewriting it during the pull).  The writer picks the buffer ON THE GPU, when the publish
  executes (ipc_kernels.hip ``ipc_param_publish``): neither the newest version's buffer nor
  any pinned one -- at most R are pinned, so one of K is always free -- marks it begun, copies,
  then releases the new word.  Once its pin is visible a reader's buffer is never rewritten,
  however slow its copy and however far the learner's host runs ahead of its GPU: publishing
  every learner iteration never starves a reader (a pull fails only if two versions are
  published between reading the word and storing the pin -- microseconds -- and is retried).
  Readers simply skip versions.
* **Liveness** (SURVEY §5.3): actors bump a heartbeat word on a wall-clock period (also
  while waiting for credit); rank 0 drops a link whose word stopped moving for
  ``dead_after`` s: its ingest mask goes to 0 and its drop flag tells a live-but-stuck actor
  to exit.  Stop = flag + acknowledgement, then rank 0 ingests until it has applied every
  packet the acknowledged actors counted as sent; nothing is ever left posted.  The control block is unlinked from /dev/shm as soon as every actor
  has mapped it.

The same code runs with every rank on ONE GPU (hipIpcOpenMemHandle in another process of
the same device), which is how the 1-GPU box exercises it.
"""
from __future__ import annotations

import ctypes
import json
import mmap
import os
import time
from datetime import timedelta

import numpy as np
import torch

from .. import ops
from .experience import META_COLS, STOP

FRAME_BYTES = 84 * 84
MODE_UNCACHED = 2

# control block layout (int64 words)
_HDR = 8          # magic, R, param word (version << 8 | buffer), stop, (reserved)
_MAGIC = 0x4150455849504331  # "APEXIPC1"


def _align(n: int, a: int = 256) -> int:
    return -(-n // a) * a


def packet_bytes(E: int) -> int:
    return E * (FRAME_BYTES + META_COLS * 4)


def param_buffers(R: int) -> int:
    """Parameter buffers of the pinned publish protocol: one per reader that may hold a pin,
    plus the newest version, plus one the writer can always take."""
    return int(R) + 2


def pick_buffer(word: int, pins, K: int) -> int:
    """Writer side of the pinned protocol (what ``ipc_param_publish`` computes on the GPU):
    the lowest buffer that is neither the current word's nor pinned by a reader (pins hold the
    words the readers pinned; 0 = none)."""
    busy = {int(word) & 0xFF} | {int(p) & 0xFF for p in pins if int(p) != 0}
    return next(b for b in range(K) if b not in busy)


def pinned_pull(ctrl: "ControlBlock", i: int, have: int, pull, retries: int = 8) -> tuple[int | None, int]:
    """Reader side of the pinned protocol for reader ``i``: pin the newest published word,
    ``pull(buffer)`` it (synchronously), keep it if the buffer's begin word still reads that
    version.  Returns (installed version or None, failed pulls)."""
    w = ctrl.param_word
    if (w >> 8) <= have:
        return None, 0
    pin = ctrl.view("pin")
    failed = 0
    try:
        for _ in range(retries):
            pin[i] = w  # from here on the writer leaves this buffer alone
            v, b = w >> 8, w & 0xFF
            pull(b)
            if int(ctrl.w[ctrl.begin_off(b)]) == v:  # nobody began rewriting it during the pull: clean
                return v, failed
            failed += 1
            w = ctrl.param_word
        return None, failed
    finally:
        pin[i] = 0


class ControlBlock:
    """int64 words in /dev/shm: header | consumed[R] | heartbeat[R] | drop[R] | sent[R] | ack[R]
    | pin[R] | begin[K] (K = param_buffers(R): the version each parameter buffer last began)."""

    FIELDS = ("consumed", "heartbeat", "drop", "sent", "ack", "pin")

    def __init__(self, name: str, R: int, create: bool):
        self.name, self.R = name, int(R)
        self.K = param_buffers(self.R)
        self.path = f"/dev/shm/{name}"
        self.nbytes = _align(8 * (_HDR + len(self.FIELDS) * self.R + self.K), 4096)
        if create:
            fd = os.open(self.path, os.O_CREAT | os.O_EXCL | os.O_RDWR, 0o600)
            os.ftruncate(fd, self.nbytes)
        else:
            fd = os.open(self.path, os.O_RDWR)
        try:
            self.mm = mmap.mmap(fd, self.nbytes)
        finally:
            os.close(fd)
        self.w = np.frombuffer(self.mm, dtype=np.int64)
        if create:
            self.w[:] = 0
            self.w[1] = self.R
            self.w[0] = _MAGIC
        elif self.w[0] != _MAGIC or self.w[1] != self.R:
            raise RuntimeError(f"{self.path}: not an apex control block for {R} links")
        self.host_ptr = ctypes.addressof(ctypes.c_char.from_buffer(self.mm))
        self.dev_ptr = None
        self._hip = None

    def off(self, field: str) -> int:
        """Word offset of ``field[0]``."""
        return _HDR + self.FIELDS.index(field) * self.R

    def view(self, field: str) -> np.ndarray:
        o = self.off(field)
        return self.w[o:o + self.R]

    def begin_off(self, b: int) -> int:
        """Word offset of parameter buffer ``b``'s begin word."""
        return _HDR + len(self.FIELDS) * self.R + int(b)

    @property
    def param_word(self) -> int:
        """The published parameter word: version << 8 | buffer."""
        return int(self.w[2])

    @property
    def param_version(self) -> int:
        return int(self.w[2]) >> 8

    @property
    def stop(self) -> bool:
        return bool(self.w[3])

    def set_stop(self) -> None:
        self.w[3] = 1

    def register(self, hip) -> int:
        """Pin + map for kernels of this process; returns the device address of word 0."""
        self._hip = hip
        self.dev_ptr = hip.host_register(self.host_ptr, self.nbytes)
        return self.dev_ptr

    def unlink(self) -> None:
        try:
            os.unlink(self.path)
        except FileNotFoundError:
            pass

    def close(self) -> None:
        if self._hip is not None and self.dev_ptr is not None:
            self._hip.host_unregister(self.host_ptr)
            self.dev_ptr = None


def aql_packet_floats(E: int, obs: int, TA: int) -> int:
    """AQL packet (structure of arrays, 4-byte words): st [E][obs] | st2 [E][obs] |
    amu [E][TA] | act [E] (i32) | rew [E] | done [E]  (ipc_kernels.hip ipc_apply_aql_k)."""
    return E * (2 * obs + TA + 3)


def aql_packet_views(buf: torch.Tensor, E: int, obs: int, TA: int) -> dict:
    """Named views of one AQL packet buffer (f32 [aql_packet_floats]): an ``AqlInsert``
    over them (C = E, cursor 0) makes the acting kernels write the packet in place."""
    o, out = 0, {}
    for name, n in (("st", E * obs), ("st2", E * obs), ("amu", E * TA), ("act", E), ("rew", E), ("done", E)):
        out[name] = buf[o:o + n]
        o += n
    out["act"] = out["act"].view(torch.int32)
    out["st"], out["st2"] = out["st"].view(E, obs), out["st2"].view(E, obs)
    out["amu"] = out["amu"].view(E, TA)
    return out


class IpcLearnerLinks:
    """Rank-0 end: the arena, the control block, the captured ingest and the publisher.

    The transport is payload-agnostic: ``tables`` holds the ingest kernel's kind-specific
    fields (``kind`` 0 = Ape-X DQN packets into per-link replay regions, 1 = AQL rows
    appended to one replay ring; see :func:`dqn_tables` / :func:`aql_tables`) and
    ``tree_write(slots, prios)`` the priority write of the rows an ingest applied (slot -1
    = nothing there)."""

    def __init__(self, R: int, D: int, E: int, P: int, store, prefix: str, device, *, packet_nbytes: int,
                 tables: dict, tree_write, cap: int | None = None, dead_after: float = 30.0,
                 mode: int = MODE_UNCACHED, log=print, open_timeout: float = 300.0):
        self.hip = h = ops.hip()
        self.R, self.D, self.E, self.P = int(R), int(D), int(E), int(P)
        self.K = param_buffers(self.R)
        self.cap = self.D if cap is None else max(1, min(int(cap), self.D))
        self.device = torch.device(device)
        self.store, self.prefix, self.log = store, prefix, log
        self.tree_write = tree_write
        self.dead_after = float(dead_after)
        self.packet_nbytes = int(packet_nbytes)
        self.pkt = _align(self.packet_nbytes)
        self.seq_off = _align(self.R * self.D * self.pkt)
        self.par_off = _align(self.seq_off + 8 * self.R * self.D)
        self.PS = _align(4 * self.P) // 4  # parameter buffer stride (floats; 256-byte aligned buffers)
        self.nbytes = self.par_off + self.K * 4 * self.PS
        self._pick = torch.zeros(1, dtype=torch.int32, device=device)  # the publish's buffer (scratch)
        self.arena = h.ipc_alloc(self.nbytes, mode)
        self.ctrl = ControlBlock(f"apex_ipc_{prefix.replace('/', '_')}_{os.getpid()}", R, create=True)
        self.ctrl.register(h)
        dev = self.device
        i64 = dict(dtype=torch.int64, device=dev)
        self.consumed = torch.zeros(R, **i64)
        self.applied_dev = torch.zeros(R, **i64)
        self.ready = torch.zeros(R, dtype=torch.int32, device=dev)
        self.prefix_dev = torch.zeros(R, dtype=torch.int32, device=dev)
        self.live_dev = torch.ones(R, dtype=torch.int32, device=dev)
        n_out = R * self.D * E  # the drain ingests up to D packets per link
        self.slots_out = torch.full((n_out,), -1, dtype=torch.int32, device=dev)
        self.prio_out = torch.zeros(n_out, dtype=torch.float32, device=dev)
        self._n_out = R * self.cap * E
        mk = lambda cap: h.make_ipc_ingest(dict(  # noqa: E731
            tables, R=R, D=D, E=E, cap=cap, packet_bytes=self.pkt, ring=self.arena, seq=self.arena + self.seq_off,
            consumed=self.consumed.data_ptr(), ready=self.ready.data_ptr(), live=self.live_dev.data_ptr(),
            prefix=self.prefix_dev.data_ptr(), host_consumed=self.ctrl.dev_ptr + 8 * self.ctrl.off("consumed"),
            applied=self.applied_dev.data_ptr(), slots_out=self.slots_out.data_ptr(),
            prio_out=self.prio_out.data_ptr()))
        self.ingest_handle = mk(self.cap)
        self.drain_handle = mk(self.D)
        self.version = 0
        self.live = set(range(1, R + 1))
        self.dropped: dict[int, str] = {}
        self._hb = {r: (None, time.monotonic()) for r in self.live}
        self._hb_t = time.monotonic()
        self.closed = False
        geo = dict(R=R, D=D, E=E, P=P, PS=self.PS, pkt=self.pkt, packet_nbytes=self.packet_nbytes, seq_off=self.seq_off,
                   par_off=self.par_off, shm=self.ctrl.name, device=self.device.index or 0)
        store.set(f"{prefix}/ipc/handle", h.ipc_handle(self.arena))
        store.set(f"{prefix}/ipc/geometry", json.dumps(geo))
        # every actor has mapped the control block -> remove its name (nothing lingers in /dev/shm)
        self._open_timeout = float(open_timeout)
        self._unlinked = False

    @classmethod
    def for_dqn(cls, R: int, D: int, E: int, P: int, replay, regions: dict, store, prefix: str, device, **kw):
        """Ape-X DQN links: packets of E new frames + E transition rows (parallel.experience
        META_COLS layout) scattered into link r's region of ``replay`` (engine.hbm_replay)."""
        dev = torch.device(device)
        i64 = dict(dtype=torch.int64, device=dev)
        fb = torch.tensor([regions[r].frame_base for r in range(1, R + 1)], **i64)
        sb = torch.tensor([regions[r].slot_base for r in range(1, R + 1)], **i64)
        rp = replay
        tables = dict(kind=0, filled=rp.filled.data_ptr(), frames=rp.frames.data_ptr(), s_ids=rp.s_ids.data_ptr(),
                      s2_ids=rp.s2_ids.data_ptr(), action=rp.action.data_ptr(), reward=rp.reward.data_ptr(),
                      done=rp.done.data_ptr(), frame_base=fb.data_ptr(), slot_base=sb.data_ptr())
        def tree_write(slots, prios):  # ring-ordered new rows (slot -1: nothing there)
            # one-workgroup fused writes (leaves + every level) of <= 4096 rows each: they run on
            # the learner's tree stream beside the conv backward, where wide per-level launches
            # slow the backward's GEMMs (profiles/r5_x6.md, learner tree branch)
            for k in range(0, slots.numel(), 4096):
                rp.write_priorities(slots[k:k + 4096], prios[k:k + 4096], dedup=False)

        links = cls(R, D, E, P, store, prefix, device, packet_nbytes=packet_bytes(E), tables=tables,
                    tree_write=tree_write, **kw)
        links.replay, links.frame_base, links.slot_base = rp, fb, sb  # (kept alive: the kernel reads them)
        return links

    @classmethod
    def for_aql(cls, R: int, D: int, E: int, P: int, replay, store, prefix: str, device, gate: tuple | None = None,
                **kw):
        """AQL links (AQL_dis.py:109-126 over xGMI): packets of E raw (s, s', a_mu, a, r, d)
        rows appended to ``replay``'s ring (engine.aql.AQLReplay) at max priority
        (CustomPrioritizedReplayBuffer_AQL.add, memory.py:368-378).  ``gate`` = (budget i64 [1],
        gate i32 [1], batch, max steps): every ingest turns the rows it applied into the SGD
        steps they pay for (kernels.h IpcIngest)."""
        rp = replay
        TA = rp.T * rp.adim
        if rp.capacity < R * D * E:  # the drain ingests up to D packets per link into the ring
            raise ValueError(f"AQL links: replay capacity {rp.capacity} < R x D x E = {R} x {D} x {E}")
        tables = dict(kind=1, obs=rp.obs, TA=TA, aql_st=rp.st.data_ptr(), aql_st2=rp.st2.data_ptr(),
                      aql_amu=rp.a_mu.data_ptr(), aql_act=rp.action.data_ptr(), aql_rew=rp.reward.data_ptr(),
                      aql_done=rp.done.data_ptr(), aql_C=rp.capacity, filled=rp.filled.data_ptr())
        if gate is not None:
            tables.update(budget=gate[0].data_ptr(), gate=gate[1].data_ptr(), gate_batch=int(gate[2]),
                          gate_max=int(gate[3]))
        h = ops.hip()

        def tree_write(slots, _prios):  # every new row at the running max priority (ring order, -1 skipped)
            h.per_write_leaves(rp.tree, slots.data_ptr(), 0, slots.numel(), rp.alpha, rp.max_prio.data_ptr(), 0, 0,
                               0, 0, 0, 0, torch.cuda.current_stream().cuda_stream)

        links = cls(R, D, E, P, store, prefix, device, packet_nbytes=4 * aql_packet_floats(E, rp.obs, TA),
                    tables=tables, tree_write=tree_write, **kw)
        links.replay = rp
        return links

    def _maybe_unlink(self) -> None:
        if self._unlinked:
            return
        keys = [f"{self.prefix}/ipc/opened/{r}" for r in range(1, self.R + 1)]
        if all(self.store.check([k]) for k in keys):
            self.ctrl.unlink()
            self._unlinked = True

    @staticmethod
    def _s() -> int:
        return torch.cuda.current_stream().cuda_stream

    def ingest(self, drain: bool = False) -> None:
        """Apply every ready packet (<= cap per link; ``drain``: <= D), release the slots,
        write the tree.  Device-only, on the current stream: capture it in the learner graph."""
        self.hip.ipc_ingest(self.drain_handle if drain else self.ingest_handle, self._s())
        n = self.slots_out.numel() if drain else self._n_out
        self.tree_write(self.slots_out[:n], self.prio_out[:n])

    def publish(self, flat: torch.Tensor) -> int:
        """Conflated versioned publish (pinned protocol, module docstring), on the current
        stream: the GPU picks a buffer neither current nor pinned when the publish executes,
        marks it begun, copies ``flat`` into it and releases the new word.  Returns the version."""
        self.version += 1
        c = self.ctrl
        self.hip.ipc_param_publish(c.dev_ptr, c.off("pin"), self.R, c.begin_off(0), self.K,
                                   self.arena + self.par_off, self.PS, flat.data_ptr(), self.P, self.version,
                                   self._pick.data_ptr(), self._s())
        return self.version

    def drop(self, r: int, why: str) -> None:
        if r in self.live:
            self.live.discard(r)
            self.dropped[r] = why
            self.live_dev[r - 1] = 0     # stream-ordered: later ingests skip the link
            self.ctrl.view("drop")[r - 1] = 1
            if self.log:
                self.log(f"[central/ipc] dropping actor rank {r}: {why}")

    def check_heartbeats(self, every: float = 1.0) -> None:
        now = time.monotonic()
        if now - self._hb_t < every:
            return
        self._hb_t = now
        self._maybe_unlink()
        hb = self.ctrl.view("heartbeat")
        for r in sorted(self.live):
            v = int(hb[r - 1])
            prev, t = self._hb[r]
            if v != prev:
                self._hb[r] = (v, now)
            elif now - t > self.dead_after:
                self.drop(r, f"no heartbeat for {self.dead_after:.0f}s")

    def applied(self) -> dict:
        """Packets applied per link (device counters; one host sync)."""
        a = self.applied_dev.tolist()
        return {r: int(a[r - 1]) for r in range(1, self.R + 1)}

    def close(self, timeout: float = 60.0) -> dict:
        """Stop every actor (flag + acknowledgement, bounded), drain what they pushed before
        acknowledging (every packet of a live link reaches the replay), release the arena."""
        if self.closed:
            return self.stats()
        self.closed = True
        torch.cuda.synchronize(self.device)
        self.ctrl.set_stop()
        ack, sent = self.ctrl.view("ack"), self.ctrl.view("sent")
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline and not all(ack[r - 1] for r in self.live):
            self.ingest(drain=True)  # keep consuming: an actor blocked on credit must see its push land
            torch.cuda.synchronize(self.device)
            time.sleep(0.001)
        for r in sorted(self.live):
            if not ack[r - 1]:
                self.drop(r, "stop not acknowledged")
        # every live actor acknowledged after its last push landed (finish() synchronises
        # first): its ``sent`` is final -- apply up to it, on a deadline of its own
        deadline = time.monotonic() + timeout
        while True:
            done = self.applied()
            short = {r: int(sent[r - 1]) - done[r] for r in sorted(self.live) if done[r] < int(sent[r - 1])}
            if not short:
                break
            if time.monotonic() > deadline:
                for r, k in short.items():  # never silent: the shortfall shows in stats()["dropped"]
                    self.drop(r, f"drain timed out with {k} pushed packets unapplied")
                break
            self.ingest(drain=True)
            torch.cuda.synchronize(self.device)
        st = self.stats()
        self.ctrl.unlink()
        self.ctrl.close()
        self.hip.ipc_free(self.arena)
        self.arena = 0
        return st

    def stats(self) -> dict:
        sent = self.ctrl.view("sent")
        return {"applied": self.applied(), "sent": {r: int(sent[r - 1]) for r in range(1, self.R + 1)},
                "dropped": dict(self.dropped), "live": sorted(self.live), "params_version": self.version,
                "transport": "hip-ipc"}


class IpcActorLink:
    """Actor end: peer copies into rank 0's ring with the credit window, pulls of the
    newest parameter version, heartbeat, drop and stop."""

    def __init__(self, rank: int, store, prefix: str, flat: torch.Tensor, packet: torch.Tensor, device,
                 heartbeat_every: float = 0.5, timeout: float = 300.0, credit_timeout: float = 120.0):
        self.hip = h = ops.hip()
        self.credit_timeout = float(credit_timeout)
        self.rank, self.store, self.prefix = rank, store, prefix
        self.device = torch.device(device)
        self.flat, self.packet = flat, packet
        store.wait([f"{prefix}/ipc/handle", f"{prefix}/ipc/geometry"], timedelta(seconds=timeout))
        geo = json.loads(store.get(f"{prefix}/ipc/geometry"))
        self.R, self.D, self.E, self.P, self.PS = geo["R"], geo["D"], geo["E"], geo["P"], geo["PS"]
        self.K = param_buffers(self.R)
        self.pkt, self.seq_off, self.par_off = geo["pkt"], geo["seq_off"], geo["par_off"]
        want = geo.get("packet_nbytes", packet_bytes(self.E))
        if packet.numel() * packet.element_size() != want or not packet.is_contiguous():
            raise ValueError(f"packet buffer must be {want} contiguous bytes (the learner's packet layout)")
        if flat.numel() != self.P:
            raise ValueError(f"parameter count {flat.numel()} != the learner's {self.P}")
        self.remote = h.ipc_open(store.get(f"{prefix}/ipc/handle"), self.device.index or 0)
        self.ctrl = ControlBlock(geo["shm"], self.R, create=False)
        store.set(f"{prefix}/ipc/opened/{rank}", "1")
        self.i = rank - 1
        self.consumed = self.ctrl.view("consumed")
        self.hb = self.ctrl.view("heartbeat")
        self.period = float(heartbeat_every)
        self._hb_t = 0.0
        self.sent = 0
        self.version = 0
        self.pulls_retried = 0
        self.stopped = False
        self.dropped = False
        self._ev = torch.cuda.Event()
        self.beat(force=True)

    @staticmethod
    def _s() -> int:
        return torch.cuda.current_stream().cuda_stream

    @property
    def n_sent(self) -> int:
        return self.sent

    def beat(self, force: bool = False) -> None:
        now = time.monotonic()
        if force or now - self._hb_t >= self.period:
            self._hb_t = now
            self.hb[self.i] += 1

    def check_stop(self) -> bool:
        """True once rank 0 has stopped or dropped this link (acknowledges a stop)."""
        if self.stopped:
            return True
        if self.ctrl.view("drop")[self.i]:
            self.dropped = True
            self.finish()
        elif self.ctrl.stop:
            self.finish()
        return self.stopped

    def push(self, timeout: float | None = None) -> bool:
        """Copy the packet into the next ring slot and publish its sequence number (both on
        the current stream, behind the actor step that filled it).  Waits (bounded) while
        ``D`` packets are unconsumed.

        The packet is already staged and the actor's local mirror already holds its rows, so
        a *stop* seen while waiting does not abandon it: rank 0 keeps draining until every
        live actor has acknowledged (IpcLearnerLinks.close), credit arrives, the packet is
        pushed and the next :meth:`check_stop` acknowledges (the reference acks every push,
        actor.py:105-115 / replay.py:94, so an accepted batch is never lost).  Only a *drop*
        abandons it (rank 0 no longer ingests this link): then False."""
        n = self.sent
        timeout = self.credit_timeout if timeout is None else float(timeout)
        deadline = time.monotonic() + timeout
        while n - int(self.consumed[self.i]) >= self.D:
            self.beat()
            if self.stopped or self.ctrl.view("drop")[self.i]:
                self.check_stop()  # a drop: acknowledge and abandon the staged packet
                return False
            if time.monotonic() > deadline:
                raise TimeoutError(f"actor rank {self.rank}: no credit for {timeout:.0f}s "
                                   f"(sent {n}, consumed {int(self.consumed[self.i])}, stop {self.ctrl.stop})")
            time.sleep(0.0001)
        k, s = n % self.D, self._s()
        slot = self.remote + (self.i * self.D + k) * self.pkt
        self.hip.memcpy_async(slot, self.packet.data_ptr(), self.packet.numel() * self.packet.element_size(), s)
        self.hip.ipc_flag(self.remote + self.seq_off + 8 * (self.i * self.D + k), n + 1, s)
        self.sent = n + 1
        self.ctrl.view("sent")[self.i] = self.sent
        self.beat()
        return True

    def poll_params(self, retries: int = 8):
        """None (nothing new), STOP, or the version just installed into ``flat`` (the
        pinned protocol's reader, module docstring)."""
        if self.check_stop():
            return STOP
        def pull(b: int) -> None:
            self.hip.memcpy_async(self.flat.data_ptr(), self.remote + self.par_off + b * 4 * self.PS, 4 * self.P,
                                  self._s())
            self._ev.record(torch.cuda.current_stream(self.device))
            self._ev.synchronize()

        v, failed = pinned_pull(self.ctrl, self.i, self.version, pull, retries)
        self.pulls_retried += failed
        if v is not None:
            self.version = v
        return v

    def finish(self) -> None:
        if self.stopped:
            return
        torch.cuda.synchronize(self.device)  # our last peer copies have landed
        self.stopped = True
        self.ctrl.view("ack")[self.i] = 1
        self.hip.ipc_close(self.remote)
        self.remote = 0


class EmulatedActorLinks:
    """R actor links emulated inside rank 0's process (``bench.py --emulate-links R``): a
    one-GPU model of the central learner's load at N = R + 1 GPUs.  Every :meth:`push` writes,
    for each link whose credit window allows it, one synthetic Ape-X packet (E frames + E rows
    at the link's next local slots) straight into the learner's IPC ring slot and then stores
    the slot's sequence word -- the bytes and the release protocol an actor GPU's xGMI peer copy
    delivers (ipc_kernels.hip ``ipc_emu_*``).  The learner side is the real one: the in-graph
    ``ipc_ingest``, the batched tree write, the credit counters, the stop / drain handshake
    (the emulated actors acknowledge a stop in :meth:`finish`)."""

    def __init__(self, links: IpcLearnerLinks, C_r: int, F_r: int, n_actions: int, seed: int = 0,
                 pool_frames: int = 4096):
        self.links, self.hip = links, links.hip
        dev = links.device
        g = torch.Generator(device=dev).manual_seed(seed)
        self.pool = torch.randint(0, 256, (pool_frames, FRAME_BYTES), dtype=torch.uint8, device=dev, generator=g)
        self.sent = torch.zeros(links.R, dtype=torch.int64, device=dev)
        self.go = torch.zeros(links.R, dtype=torch.int32, device=dev)
        self.handle = self.hip.make_ipc_emu(dict(
            ring=links.arena, seq=links.arena + links.seq_off, consumed=links.consumed.data_ptr(),
            sent=self.sent.data_ptr(), go=self.go.data_ptr(), pool=self.pool.data_ptr(), pool_n=pool_frames,
            R=links.R, D=links.D, E=links.E, C_r=int(C_r), F_r=int(F_r), n_actions=int(n_actions), pkt=links.pkt,
            seed=(seed * 0x9E3779B97F4A7C15 + 1) & 0xFFFFFFFFFFFFFFFF))
        for r in range(1, links.R + 1):  # every "actor" has mapped the control block
            links.store.set(f"{links.prefix}/ipc/opened/{r}", "1")
        self._hb = links.ctrl.view("heartbeat")

    def push(self) -> None:
        """One paced actor step of every link (credit permitting), on the current stream."""
        self.hip.ipc_emu_push(self.handle, torch.cuda.current_stream().cuda_stream)
        self._hb += 1  # alive

    def finish(self) -> None:
        """Acknowledge the stop: the final sent counts, then the acks (the learner drains them)."""
        torch.cuda.synchronize(self.links.device)
        self.links.ctrl.view("sent")[:] = self.sent.cpu().numpy()
        self.links.ctrl.view("ack")[:] = 1
