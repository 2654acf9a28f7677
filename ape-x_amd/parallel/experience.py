"""Asynchronous actor -> learner experience links for the central-replay topology
(reference actor.py:40-49,105-115, replay.py:77-146,
learner.py:57-68).

Rank 0 owns the single HBM replay and the learner; ranks 1..W-1 run GPU actor shards.
Each actor rank writes into a *local mirror* of its region of the rank-0 replay (same
frame-ring and transition-slot geometry), so one actor step produces, at positions the
shard itself reports, E new frames and E transition rows (priority 0 = no row).  A
*packet* is one actor step: frames ``[E, frame_bytes]`` u8 + metadata ``[E, 14]`` i32.

Transport (one torch.distributed P2P group per actor link, so a slow or dead link never
blocks another: with ``nccl`` each link has its own RCCL communicator / stream over xGMI,
with ``gloo`` packets are staged through pinned host memory):

* :class:`PacketSender` (actor): a ring of ``depth`` packet slots; at most ``depth``
  packets in flight -- the reference's credit window (actor.py:105-115 keeps 3 pushes
  outstanding).  Acquiring a slot waits (bounded) for its previous send.
* :class:`PacketInbox` (rank 0): ``depth`` receives always pre-posted; :meth:`poll` hands
  back the packets that have landed, in send order, without blocking; a failed receive
  (peer gone) marks the link dead.
* :func:`apply_packets`: every ready packet of every link scattered into its region and
  written into the priority tree as ONE batch of device ops between learner steps (no
  per-round host ``take()``, no lock-step).
* :class:`ParamLink` / :class:`ParamSubscriber`: conflated, versioned parameter publish
  (reference PUB/SUB with CONFLATE, actor.py:40-49): rank 0 sends the newest snapshot to
  a link only when that link's previous snapshot has been delivered; version -1 = stop.
* :class:`Heartbeats`: actors bump a time-driven beat counter in the TCPStore (also while
  blocked on credit); rank 0 drops a link whose counter has not moved for ``dead_after``
  seconds and sets ``<prefix>/drop/<r>``, which a still-running actor sees and exits 0 on
  (SURVEY §5.3).  Every key carries a per-engine nonce prefix (:func:`engine_nonce`).
* Each link has two P2P groups (:class:`LinkGroups`): packets and parameters never share
  an RCCL stream.

Shutdown handshake (bounded, see ``CentralApexEngine.close``): rank 0 sends stop on the
param channel; the actor publishes its packet count; rank 0 publishes how many packets
it has receives posted for; the actor pads with dummy packets (slot -1) until the two
match, so no receive or send is left dangling.
"""
from __future__ import annotations

import queue
import threading
import time
from datetime import timedelta

import torch
import torch.distributed as dist

META_COLS = 14
STOP = -1


def pack_meta(s_ids, s2_ids, action, reward, done, prio, slot, fslot, out: torch.Tensor | None = None):
    """[E, 14] int32 packing of one actor step (floats as raw bits): s_ids 4 | s2_ids 4 |
    action | reward | done | priority | local transition slot | local new-frame slot.
    Pure device ops (graph-capturable)."""
    E = action.numel()
    out = out if out is not None else torch.empty(E, META_COLS, dtype=torch.int32, device=action.device)
    out[:, 0:4].copy_(s_ids.reshape(E, 4))
    out[:, 4:8].copy_(s2_ids.reshape(E, 4))
    out[:, 8].copy_(action.reshape(E))
    out[:, 9].copy_(reward.reshape(E).contiguous().view(torch.int32))
    out[:, 10].copy_(done.reshape(E).contiguous().view(torch.int32))
    out[:, 11].copy_(prio.reshape(E).contiguous().view(torch.int32))
    out[:, 12].copy_(slot.reshape(E))
    out[:, 13].copy_(fslot.reshape(E))
    return out


class Region:
    """Where remote rank r's experience lives inside the rank-0 replay."""

    def __init__(self, slot_base: int, n_slots: int, frame_base: int, n_frames: int):
        self.slot_base, self.n_slots = int(slot_base), int(n_slots)
        self.frame_base, self.n_frames = int(frame_base), int(n_frames)


def apply_packet(tables: dict, region: Region, frames: torch.Tensor, meta: torch.Tensor):
    """Write one remote actor step into region ``region`` of the rank-0 tables; returns
    (global slots int32 [E], priorities f32 [E]) for the priority-tree write."""
    fslot = meta[:, 13].long() + region.frame_base
    tables["frames"].index_copy_(0, fslot, frames)
    slot = meta[:, 12].long() + region.slot_base
    ids = meta[:, 0:8] + region.frame_base
    tables["s_ids"].index_copy_(0, slot, ids[:, 0:4].contiguous())
    tables["s2_ids"].index_copy_(0, slot, ids[:, 4:8].contiguous())
    tables["action"].index_copy_(0, slot, meta[:, 8].contiguous())
    tables["reward"].index_copy_(0, slot, meta[:, 9].contiguous().view(torch.float32))
    tables["done"].index_copy_(0, slot, meta[:, 10].contiguous().view(torch.float32))
    return slot.to(torch.int32), meta[:, 11].contiguous().view(torch.float32)


def apply_packets(tables: dict, frames: torch.Tensor, meta: torch.Tensor, frame_base: torch.Tensor,
                  slot_base: torch.Tensor):
    """Batched :func:`apply_packet`: ``frames`` [n, E, FB], ``meta`` [n, E, 14] (n ready
    packets, any links), ``frame_base`` / ``slot_base`` int64 [n] the packets' region
    offsets.  One set of scatters for all packets; returns (slots int32, priorities)."""
    n, E = meta.shape[0], meta.shape[1]
    m = meta.reshape(n * E, META_COLS)
    fb = frame_base.repeat_interleave(E)
    sb = slot_base.repeat_interleave(E)
    tables["frames"].index_copy_(0, m[:, 13].long() + fb, frames.reshape(n * E, -1))
    local = m[:, 12].long()
    slot = local + sb
    real = local >= 0  # filler rows (slot -1, e.g. the reset-frame packet) carry frames only
    ids = m[:, 0:8] + fb.to(torch.int32).unsqueeze(1)
    rows = (ids[:, 0:4], ids[:, 4:8], m[:, 8], m[:, 9].contiguous().view(torch.float32),
            m[:, 10].contiguous().view(torch.float32))
    if not bool(real.all()):  # eager path only (host-staged links): a data-dependent subset
        keep = real.nonzero().squeeze(1)
        rows = tuple(t.index_select(0, keep) for t in rows)
        dst = slot.index_select(0, keep)
    else:
        dst = slot
    for name, t in zip(("s_ids", "s2_ids", "action", "reward", "done"), rows):
        tables[name].index_copy_(0, dst, t.contiguous())
    return torch.where(real, slot, -1).to(torch.int32), m[:, 11].contiguous().view(torch.float32)


def _via_host(device: torch.device, group) -> bool:
    return device.type == "cuda" and dist.get_backend(group) != "nccl"


class _Pending:
    __slots__ = ("works", "event", "error")

    def __init__(self, works):
        self.works, self.event, self.error = works, threading.Event(), None


class WorkTracker:
    """Completion of torch.distributed P2P works without blocking the caller.  RCCL/NCCL
    works report ``is_completed()`` (event query).  Gloo P2P works only complete inside
    ``wait()``, so a daemon thread per channel waits on them in posting order (the GIL is
    released while it blocks) and flags each batch; a failed wait (peer gone) is recorded
    and re-raised by :meth:`done`."""

    def __init__(self, group):
        self.native = dist.get_backend(group) == "nccl"
        self.q: queue.Queue | None = None

    def add(self, works) -> _Pending:
        p = _Pending(works)
        if not self.native:
            self._queue().put(p)
        return p

    def add_deferred(self, event, issue) -> _Pending:
        """Gloo only: the tracker thread waits for ``event`` (e.g. the D2H copy that filled
        the send buffer), then calls ``issue()`` for the works and waits for them."""
        assert not self.native
        p = _Pending((event, issue))
        self._queue().put(p)
        return p

    def _queue(self) -> queue.Queue:
        if self.q is None:
            self.q = queue.Queue()
            threading.Thread(target=self._run, args=(self.q,), daemon=True).start()
        return self.q

    @staticmethod
    def _run(q):
        while True:
            p = q.get()
            try:
                if isinstance(p.works, tuple):  # deferred issue
                    ev, issue = p.works
                    ev.synchronize()
                    p.works = issue()
                for w in p.works:
                    w.wait()
            except Exception as e:  # recorded for the poller
                p.error = e
            finally:
                p.event.set()

    def done(self, p: _Pending | None) -> bool:
        if p is None:
            return True
        if self.native:
            return all(w.is_completed() for w in p.works)
        if p.error is not None:
            raise p.error
        return p.event.is_set()

    def wait(self, p: _Pending | None, timeout: float) -> bool:
        """Bounded wait: True when completed (an error raises)."""
        deadline = time.monotonic() + timeout
        while not self.done(p):
            if time.monotonic() > deadline:
                return False
            time.sleep(0.0002)
        if p is not None and self.native:
            for w in p.works:
                w.wait()  # orders the caller's stream after the transfer (no host block)
        return True


class LinkGroups:
    """The two P2P channels of one actor link, each on its own group: with ``nccl`` every
    group is its own RCCL communicator *and stream*, so a receive posted on one channel
    (the actor's parameter subscription, rank 0's pre-posted packet receives) never sits
    in front of traffic on the other.  One shared group deadlocks: the actor's first
    packet would queue behind its posted parameter receive, which waits for a publish
    that waits for that packet."""

    __slots__ = ("packets", "params")

    def __init__(self, packets, params):
        self.packets, self.params = packets, params


def link_groups(world: int) -> dict:
    """{r: LinkGroups} for every actor rank r; collective: every rank calls it (same order)."""
    return {r: LinkGroups(dist.new_group([0, r]), dist.new_group([0, r])) for r in range(1, world)}


def engine_nonce(store) -> str:
    """A key prefix unique to this engine instance (rank 0 draws it from the store, every
    rank learns it through a broadcast; collective): a second engine on the same store
    never reads the handshake / heartbeat keys of an earlier one."""
    box = [int(store.add("apex/engine_gen", 1)) if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(box, src=0)
    return f"apex/{box[0]}"


class PacketSender:
    """Actor end of a link: ``depth`` packet slots, at most ``depth`` in flight."""

    def __init__(self, E: int, frame_bytes: int, device, group, dst: int = 0, depth: int = 3):
        self.device = torch.device(device)
        self.group, self.dst, self.depth = group, dst, int(depth)
        self.via_host = _via_host(self.device, group)
        dev = "cpu" if self.via_host else self.device
        pin = self.via_host and torch.cuda.is_available()
        mk = lambda *s, dt: (torch.empty(*s, dtype=dt).pin_memory() if pin else  # noqa: E731
                             torch.empty(*s, dtype=dt, device=dev))
        self.frames = [mk(E, frame_bytes, dt=torch.uint8) for _ in range(depth)]
        self.meta = [mk(E, META_COLS, dt=torch.int32) for _ in range(depth)]
        self.works: list = [None] * depth
        self.track = WorkTracker(group)
        self.k = 0
        self.n_sent = 0

    def acquire(self, timeout: float = 60.0, on_wait=None, every: float = 0.25):
        """(frames, meta) buffers of the next slot, once its previous send has left
        (credit window).  ``on_wait()`` runs every ``every`` s while blocked (heartbeat,
        drop check; it may raise).  Raises TimeoutError if the learner stopped draining."""
        deadline = time.monotonic() + timeout
        while not self.track.wait(self.works[self.k], every if on_wait else timeout):
            if time.monotonic() > deadline:
                raise TimeoutError(f"experience link to rank {self.dst}: no credit for {timeout}s")
            if on_wait is not None:
                on_wait()
        self.works[self.k] = None
        return self.frames[self.k], self.meta[self.k]

    def send(self) -> None:
        k = self.k
        if self.via_host and torch.cuda.is_available():
            # host-staged (gloo): the slot was filled by a D2H copy on the caller's stream; the
            # tracker thread waits for that copy's event before handing the slot to gloo, so
            # the actor's host thread never blocks on its own GPU work
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self.works[k] = self.track.add_deferred(ev, lambda k=k: [
                dist.isend(self.frames[k], self.dst, group=self.group),
                dist.isend(self.meta[k], self.dst, group=self.group)])
        else:
            self.works[k] = self.track.add([dist.isend(self.frames[k], self.dst, group=self.group),
                                            dist.isend(self.meta[k], self.dst, group=self.group)])
        self.k = (k + 1) % self.depth
        self.n_sent += 1

    def send_dummy(self, timeout: float = 60.0) -> None:
        """A filler packet (slot -1): matches one receive the learner has posted."""
        _, meta = self.acquire(timeout)
        meta.fill_(-1)
        self.send()

    def drain(self, timeout: float = 60.0) -> bool:
        ok = True
        for i in range(self.depth):
            ok = self.track.wait(self.works[i], timeout) and ok
            self.works[i] = None
        return ok


class PacketInbox:
    """Learner end of a link: ``depth`` receives pre-posted into ``frames`` / ``meta``
    ([depth, E, ...]); packets complete in send order."""

    def __init__(self, src: int, frames: torch.Tensor, meta: torch.Tensor, group, device):
        self.src, self.group = src, group
        self.device = torch.device(device)
        self.via_host = _via_host(self.device, group)
        self.depth = frames.shape[0]
        self.dev_frames, self.dev_meta = frames, meta  # device views (the batched apply reads these)
        if self.via_host:
            # 2*depth pinned host buffers, rotated per packet: a packet's H2D copy is issued
            # non-blocking on the learner stream and its buffer is re-armed only once that copy's
            # event has completed (two packets later), so the host never waits on the GPU
            pin = torch.cuda.is_available()
            nb = 2 * self.depth
            mk = lambda t: torch.empty((nb,) + tuple(t.shape[1:]), dtype=t.dtype)  # noqa: E731
            self.frames, self.meta = mk(frames), mk(meta)
            if pin:
                self.frames, self.meta = self.frames.pin_memory(), self.meta.pin_memory()
            self.h_event = [None] * nb
        else:
            self.frames, self.meta = frames, meta
        self.works: list = [None] * self.depth
        self.hslot = [0] * self.depth  # host buffer of the receive posted into device slot k
        self.track = WorkTracker(group)
        self.n_posted = self.n_done = 0
        self.dead = False
        self.error: str | None = None

    def _post(self, k: int) -> None:
        if self.via_host:
            hb = self.n_posted % (2 * self.depth)
            if self.h_event[hb] is not None:
                self.h_event[hb].synchronize()  # (normally long done) the buffer's last H2D copy
                self.h_event[hb] = None
            self.hslot[k] = hb
            src_f, src_m = self.frames[hb], self.meta[hb]
        else:
            src_f, src_m = self.frames[k], self.meta[k]
        self.works[k] = self.track.add([dist.irecv(src_f, self.src, group=self.group),
                                        dist.irecv(src_m, self.src, group=self.group)])
        self.n_posted += 1

    def start(self) -> None:
        for k in range(self.depth):
            self._post(k)

    def poll(self, limit: int | None = None) -> list[int]:
        """Slots whose packets have landed, oldest first (non-blocking; stops at the first
        incomplete receive, so order is preserved)."""
        out = []
        if self.dead:
            return out
        k = self.n_done % self.depth
        while self.works[k] is not None and (limit is None or len(out) < limit):
            try:
                if not self.track.done(self.works[k]):
                    break
                if self.track.native:
                    for w in self.works[k].works:
                        w.wait()  # the current stream is ordered after the receive
            except Exception as e:  # the peer is gone (connection closed / comm error)
                self.dead, self.error = True, repr(e)
                break
            self.works[k] = None
            if self.via_host:  # pinned host packet -> device slot, async on the caller's stream
                hb = self.hslot[k]
                self.dev_frames[k].copy_(self.frames[hb], non_blocking=True)
                self.dev_meta[k].copy_(self.meta[hb], non_blocking=True)
                if torch.cuda.is_available() and self.dev_frames.is_cuda:
                    ev = torch.cuda.Event()
                    ev.record(torch.cuda.current_stream(self.dev_frames.device))
                    self.h_event[hb] = ev
            out.append(k)
            self.n_done += 1
            k = self.n_done % self.depth
        return out

    def repost(self, k: int, limit: int | None = None) -> None:
        """Re-arm slot ``k`` (after its packet was applied) unless ``limit`` receives
        have been posted in total."""
        if not self.dead and (limit is None or self.n_posted < limit):
            try:
                self._post(k)
            except Exception as e:  # the peer died after its last packet landed: gloo's irecv
                self.dead, self.error = True, repr(e)  # raises at post time ("Connection closed")


class ParamLink:
    """Rank-0 end of a link's parameter channel: conflated, versioned snapshots."""

    def __init__(self, flat: torch.Tensor, dst: int, group):
        self.dst, self.group = dst, group
        self.via_host = _via_host(flat.device, group)
        pin = self.via_host and torch.cuda.is_available()
        self.snap = torch.empty(flat.numel(), dtype=flat.dtype).pin_memory() if pin else \
            torch.empty(flat.numel(), dtype=flat.dtype, device="cpu" if self.via_host else flat.device)
        self.ver = torch.zeros(1, dtype=torch.int64, device="cpu" if self.via_host else flat.device)
        self.works = None
        self.track = WorkTracker(group)
        self.version = -2  # last version handed to the transport
        self.skipped = 0

    def publish(self, flat: torch.Tensor, version: int) -> bool:
        """Send ``flat`` as ``version`` if the previous snapshot was delivered (conflation:
        a busy link just gets a newer version later).  True if sent."""
        if not self.track.done(self.works):
            self.skipped += 1
            return False
        self.snap.copy_(flat.reshape(-1), non_blocking=True)
        self.ver.fill_(version)
        if self.via_host and torch.cuda.is_available():  # gloo: send once the D2H snapshot landed
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(flat.device))
            self.works = self.track.add_deferred(ev, lambda: [dist.isend(self.ver, self.dst, group=self.group),
                                                              dist.isend(self.snap, self.dst, group=self.group)])
        else:
            self.works = self.track.add([dist.isend(self.ver, self.dst, group=self.group),
                                         dist.isend(self.snap, self.dst, group=self.group)])
        self.version = version
        return True

    def done(self) -> bool:
        return self.track.done(self.works)

    def send_stop(self) -> None:
        """Issue the stop message (version -1); the previous message must be delivered."""
        self.ver.fill_(STOP)
        self.works = self.track.add([dist.isend(self.ver, self.dst, group=self.group),
                                     dist.isend(self.snap, self.dst, group=self.group)])


class ParamSubscriber:
    """Actor end of the parameter channel: one receive always posted into a staging
    buffer; :meth:`poll` swaps the newest version into ``flat``."""

    def __init__(self, flat: torch.Tensor, src: int, group):
        self.flat, self.src, self.group = flat, src, group
        self.via_host = _via_host(flat.device, group)
        dev = "cpu" if self.via_host else flat.device
        self.stage = torch.empty(flat.numel(), dtype=flat.dtype, device=dev)
        self.ver = torch.zeros(1, dtype=torch.int64, device=dev)
        self.version = 0
        self.works = None
        self.track = WorkTracker(group)
        self._post()

    def _post(self) -> None:
        self.works = self.track.add([dist.irecv(self.ver, self.src, group=self.group),
                                     dist.irecv(self.stage, self.src, group=self.group)])

    def poll(self):
        """None (nothing new), STOP, or the version just installed."""
        if self.works is None or not self.track.done(self.works):
            return None
        self.track.wait(self.works, 0.0)
        v = int(self.ver.item())
        if v == STOP:
            self.works = None
            return STOP
        self.flat.copy_(self.stage.to(self.flat.device, non_blocking=False).view_as(self.flat))
        self.version = v
        self._post()
        return v


class Heartbeats:
    """Liveness through the rendezvous TCPStore (off the data path).  An actor bumps a beat
    counter on a wall-clock period -- also while it waits for credit, so a rank-0 pause
    (graph capture, a checkpoint) never makes healthy, blocked actors look dead; rank 0
    drops a link whose counter has not moved for ``dead_after`` seconds of its own clock
    (only changes are compared, so host clocks need not agree)."""

    def __init__(self, store, ranks, dead_after: float = 30.0, prefix: str = "apex/hb", period: float = 0.5):
        self.store, self.prefix, self.dead_after = store, prefix, float(dead_after)
        self.period = float(period)
        now = time.monotonic()
        self.last = {r: (None, now) for r in ranks}
        self._count, self._t = 0, 0.0

    def beat(self, rank: int, force: bool = False) -> None:
        now = time.monotonic()
        if force or now - self._t >= self.period:
            self._t = now
            self._count += 1
            self.store.set(f"{self.prefix}/{rank}", str(self._count))

    def stale(self, ranks) -> list[int]:
        out, now = [], time.monotonic()
        for r in ranks:
            key = f"{self.prefix}/{r}"
            v = self.store.get(key) if self.store.check([key]) else None  # check: non-blocking
            prev, t = self.last[r]
            if v != prev:
                self.last[r] = (v, now)
            elif now - t > self.dead_after:
                out.append(r)
        return out


class Dropped(RuntimeError):
    """Raised on an actor whose link rank 0 has dropped (it should exit cleanly)."""


class LearnerLinks:
    """Rank-0 side of every actor link: pre-posted packet receives, conflated parameter
    publish, heartbeats, dropping dead links and the bounded stop handshake.  Landed
    packets are handed to ``apply(ready)`` as ``[(rank, ring slot)]`` with their data in
    ``frames[rank - 1, slot]`` / ``meta[rank - 1, slot]`` (device tensors)."""

    def __init__(self, world: int, groups: dict, store, flat: torch.Tensor, frames: torch.Tensor,
                 meta: torch.Tensor, apply, dead_after: float = 30.0, log=print, prefix: str = "apex"):
        self.store, self.apply_fn, self.log, self.prefix = store, apply, log, prefix
        self.frames, self.meta = frames, meta
        dev = frames.device
        self.inbox = {r: PacketInbox(r, frames[r - 1], meta[r - 1], groups[r].packets, dev) for r in range(1, world)}
        for ib in self.inbox.values():
            ib.start()
        self.params = {r: ParamLink(flat, r, groups[r].params) for r in range(1, world)}
        self.hb = Heartbeats(store, range(1, world), dead_after, prefix=f"{prefix}/hb")
        self.live = set(range(1, world))
        self.dropped: dict[int, str] = {}
        self.applied = {r: 0 for r in range(1, world)}
        self.sent: dict[int, int] = {}  # packets each actor reported sending (stop handshake)
        self.version = 0
        self._hb_t = time.monotonic()
        self.closed = False

    def drop(self, r: int, why: str) -> None:
        if r in self.live:
            self.live.discard(r)
            self.dropped[r] = why
            self.inbox[r].dead = True
            try:  # tell a still-running actor to stop (it polls this key and exits 0)
                self.store.set(f"{self.prefix}/drop/{r}", why[:200])
            except Exception:
                pass
            if self.log:
                self.log(f"[central] dropping actor rank {r}: {why}")

    def ingest(self, cap: int | None = None) -> int:
        """Apply the packets that have landed on the live links (at most ``cap`` per link:
        with the senders' credit window this paces each actor at ``cap`` packets per call,
        the reference's flow control); non-blocking."""
        ready = []
        for r in sorted(self.live):
            ib = self.inbox[r]
            ready += [(r, k) for k in ib.poll(limit=cap)]
            if ib.dead:
                self.drop(r, f"receive failed: {ib.error}")
        if ready:
            self.apply_fn(ready)
            for r, k in ready:
                self.applied[r] += 1
                self.inbox[r].repost(k)
                if self.inbox[r].dead:
                    self.drop(r, f"re-posting a receive failed: {self.inbox[r].error}")
        return len(ready)

    def check_heartbeats(self, every: float = 1.0) -> None:
        now = time.monotonic()
        if now - self._hb_t < every:
            return
        self._hb_t = now
        for r in self.hb.stale(sorted(self.live)):
            self.drop(r, f"no heartbeat for {self.hb.dead_after:.0f}s")

    def publish(self, flat: torch.Tensor) -> None:
        self.version += 1
        for r in sorted(self.live):
            try:
                self.params[r].publish(flat, self.version)
            except Exception as e:
                self.drop(r, f"param publish failed: {e!r}")

    def close(self, timeout: float = 60.0) -> dict:
        """Stop handshake with every live link (see the module docstring); bounded."""
        if self.closed:
            return self.stats()
        self.closed = True
        # deliver stop on every live link while still consuming packets: an actor blocked on
        # its credit window only re-arms its parameter receive after its next push went out
        stopping, sent_stop = set(self.live), set()
        deadline = time.monotonic() + timeout
        while stopping and time.monotonic() < deadline:
            self.ingest()
            for r in sorted(stopping):
                pl = self.params[r]
                try:
                    if not pl.done():
                        continue
                    if r in sent_stop:
                        stopping.discard(r)
                    else:
                        pl.send_stop()
                        sent_stop.add(r)
                except Exception as e:
                    self.drop(r, f"stop failed: {e!r}")
                    stopping.discard(r)
            stopping &= self.live
            time.sleep(0.0005)
        for r in sorted(stopping):
            self.drop(r, "stop not delivered")
        for r in sorted(self.live):
            ib = self.inbox[r]
            try:
                self.store.wait([f"{self.prefix}/sent/{r}"], timedelta(seconds=timeout))
                sent = int(self.store.get(f"{self.prefix}/sent/{r}"))
                self.sent[r] = sent
            except Exception as e:
                self.drop(r, f"no packet count: {e!r}")
                continue
            need = max(ib.n_posted, sent)
            self.store.set(f"{self.prefix}/need/{r}", str(need))
            deadline = time.monotonic() + timeout
            while ib.n_done < need and not ib.dead and time.monotonic() < deadline:
                ks = ib.poll()
                # filler packets are all -1 (no frame slot either; the reset-frame packet has frames)
                real = [(r, k) for k in ks if int(self.meta[r - 1, k, 0, 13].item()) >= 0]
                if real:
                    self.apply_fn(real)
                    self.applied[r] += len(real)
                for k in ks:
                    ib.repost(k, limit=need)
                if not ks:
                    time.sleep(0.0005)
            if ib.n_done < need:
                self.drop(r, "drain timed out")
        return self.stats()

    def stats(self) -> dict:
        return {"applied": dict(self.applied), "sent": dict(self.sent), "dropped": dict(self.dropped),
                "live": sorted(self.live), "params_skipped": {r: p.skipped for r, p in self.params.items()},
                "transport": "p2p"}


class ActorLink:
    """Actor side of one link: packet send ring (credit window) on the packet channel,
    parameter subscription on the parameter channel, time-driven heartbeat, the drop
    signal and the stop handshake."""

    def __init__(self, rank: int, groups: LinkGroups, store, flat: torch.Tensor, E: int, frame_bytes: int,
                 depth: int = 3, heartbeat_every: float = 0.5, prefix: str = "apex"):
        self.rank, self.store, self.prefix = rank, store, prefix
        self.sender = PacketSender(E, frame_bytes, flat.device, groups.packets, dst=0, depth=depth)
        self.sub = ParamSubscriber(flat, 0, groups.params)
        self.hb = Heartbeats(store, [], prefix=f"{prefix}/hb", period=heartbeat_every)
        self.hb.beat(rank, force=True)
        self._drop_key = f"{prefix}/drop/{rank}"
        self._drop_t = 0.0
        self.stopped = False
        self.dropped = False
        self.steps = 0

    @property
    def n_sent(self) -> int:
        return self.sender.n_sent

    def poll_params(self):
        """None / the newly installed version / STOP (after which the handshake has run)."""
        v = self.sub.poll()
        if v == STOP:
            self.finish()
        return v

    def check_dropped(self, every: float = 0.5) -> bool:
        """True once rank 0 has dropped this link (checked at most every ``every`` s)."""
        now = time.monotonic()
        if not self.dropped and now - self._drop_t >= every:
            self._drop_t = now
            self.dropped = bool(self.store.check([self._drop_key]))
        return self.dropped

    def _waiting(self) -> None:
        self.hb.beat(self.rank)
        if self.check_dropped(every=0.0):
            raise Dropped(f"actor rank {self.rank}: dropped by the learner "
                          f"({self.store.get(self._drop_key).decode(errors='replace')})")

    def push(self, frames: torch.Tensor, meta: torch.Tensor, timeout: float = 120.0) -> None:
        """Send one packet; raises :class:`Dropped` if rank 0 dropped this link meanwhile."""
        f, m = self.sender.acquire(timeout, on_wait=self._waiting)
        f.copy_(frames, non_blocking=True)  # host-staged: the send waits for this copy's event
        m.copy_(meta, non_blocking=True)
        self.sender.send()
        self.steps += 1
        self.hb.beat(self.rank)

    def finish(self, timeout: float = 120.0) -> None:
        r = self.rank
        self.store.set(f"{self.prefix}/sent/{r}", str(self.sender.n_sent))
        self.store.wait([f"{self.prefix}/need/{r}"], timedelta(seconds=timeout))
        need = int(self.store.get(f"{self.prefix}/need/{r}"))
        while self.sender.n_sent < need:
            self.sender.send_dummy(timeout)
        self.sender.drain(timeout)
        self.stopped = True
