"""Message framing for the role processes (replaces origin ZMQ + pickle).

Every message is two ``torch.distributed`` point-to-point transfers between a fixed
pair of ranks: a fixed ``int64[8]`` header ``[kind, nbytes, a0..a5]`` and, when
``nbytes > 0``, a ``uint8`` payload.  Payloads are a self-describing array bundle
(a JSON table of name/dtype/shape/offset followed by the raw bytes) -- no pickle, so
a peer can never make the receiver execute code.

Tags separate the streams a pair of ranks can have in flight at once:
``TAG_REQ`` (client -> server requests), ``TAG_REP`` (server -> client replies).
"""
from __future__ import annotations

import json

import numpy as np
import torch
import torch.distributed as dist

HEADER_LEN = 8

# message kinds
PUSH = 1          # actor -> replay: experience chunk (+ new frames)
ACK = 2           # replay -> actor
SAMPLE = 3        # learner -> replay: request a batch (a0 = batch size, a1 = beta * 1e6)
BATCH = 4         # replay -> learner
NOT_READY = 5     # replay -> learner: below threshold (a0 = current size)
PRIOS = 6         # learner -> replay: priority update
BYE = 7           # any -> replay: peer leaving
STATS = 8         # learner -> replay: ask for stats

TAG_REQ = 11
TAG_REP = 12


def pack(arrays: dict) -> np.ndarray:
    """dict[str, ndarray] -> one uint8 buffer."""
    table, chunks, off = {}, [], 0
    for k, v in arrays.items():
        a = np.ascontiguousarray(v)
        table[k] = [a.dtype.str, list(a.shape), off, a.nbytes]
        chunks.append(a.view(np.uint8).reshape(-1))
        off += a.nbytes
    head = json.dumps(table).encode()
    out = np.empty(8 + len(head) + off, dtype=np.uint8)
    out[:8] = np.frombuffer(np.int64(len(head)).tobytes(), dtype=np.uint8)
    out[8:8 + len(head)] = np.frombuffer(head, dtype=np.uint8)
    pos = 8 + len(head)
    for c in chunks:
        out[pos:pos + c.size] = c
        pos += c.size
    return out


def unpack(buf) -> dict:
    """Inverse of :func:`pack` (arrays are views into ``buf``)."""
    b = buf.numpy() if isinstance(buf, torch.Tensor) else np.asarray(buf)
    hlen = int(b[:8].view(np.int64)[0])
    table = json.loads(bytes(b[8:8 + hlen]).decode())
    base = 8 + hlen
    out = {}
    for k, (dt, shape, off, nbytes) in table.items():
        dtype = np.dtype(dt)
        if dtype.hasobject:
            raise ValueError("object arrays are not allowed on the wire")
        out[k] = b[base + off:base + off + nbytes].view(dtype).reshape(shape)
    return out


def header(kind: int, nbytes: int = 0, *args: int) -> torch.Tensor:
    h = torch.zeros(HEADER_LEN, dtype=torch.int64)
    h[0], h[1] = int(kind), int(nbytes)
    for i, a in enumerate(args[:HEADER_LEN - 2]):
        h[2 + i] = int(a)
    return h


def send_msg(dst: int, kind: int, arrays: dict | None = None, *args: int, tag: int = TAG_REQ) -> None:
    payload = pack(arrays) if arrays else None
    dist.send(header(kind, 0 if payload is None else payload.size, *args), dst, tag=tag)
    if payload is not None:
        dist.send(torch.from_numpy(payload), dst, tag=tag)


def isend_msg(dst: int, kind: int, arrays: dict | None = None, *args: int, tag: int = TAG_REQ) -> list:
    """Non-blocking send; keep the returned works (and their tensors) alive until waited."""
    payload = pack(arrays) if arrays else None
    h = header(kind, 0 if payload is None else payload.size, *args)
    works = [(dist.isend(h, dst, tag=tag), h)]
    if payload is not None:
        t = torch.from_numpy(payload)
        works.append((dist.isend(t, dst, tag=tag), t))
    return works


def recv_payload(src: int, nbytes: int, tag: int) -> dict:
    buf = torch.empty(int(nbytes), dtype=torch.uint8)
    dist.recv(buf, src, tag=tag)
    return unpack(buf)


def recv_msg(src: int, tag: int = TAG_REP):
    """Blocking receive of (header list, arrays or None) from ``src``."""
    h = torch.zeros(HEADER_LEN, dtype=torch.int64)
    dist.recv(h, src, tag=tag)
    hl = h.tolist()
    arrays = recv_payload(src, hl[1], tag) if hl[1] > 0 else None
    return hl, arrays
