"""Dependency-free TensorBoard event-file writer (tensorboardX is not installed).

Implements the TFRecord framing (u64 length, masked CRC32C of the length, payload,
masked CRC32C of the payload) around hand-encoded ``Event`` protobufs
(wall_time=1, step=2, file_version=3, summary=5 -> Summary.value=1 ->
Value{tag=1, simple_value=2}).  ``SummaryWriter(comment=...)`` writes under
``runs/<date>_<host><comment>`` exactly like tensorboardX, so the reference's
scalar tags (``learner/loss``, ``learner/grad_norm``, ``learner/BPS``,
``actor/episode_reward`` ...) show up in stock TensorBoard.
Every scalar is also mirrored to ``scalars.jsonl`` in the same directory.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import threading
import time
from datetime import datetime


def _make_crc32c_table():
    poly = 0x82F63B78
    table = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        table.append(c)
    return table


_CRC_TABLE = _make_crc32c_table()


def crc32c(data: bytes) -> int:
    crc = 0xFFFFFFFF
    t = _CRC_TABLE
    for b in data:
        crc = t[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    crc = crc32c(data)
    return (((crc >> 15) | (crc << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _len_field(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def encode_scalar_event(tag: str, value: float, step: int, wall_time: float) -> bytes:
    val = _len_field(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(value))
    summary = _len_field(1, val)
    return _key(1, 1) + struct.pack("<d", wall_time) + _key(2, 0) + _varint(int(step)) + _len_field(5, summary)


def encode_version_event(wall_time: float) -> bytes:
    return _key(1, 1) + struct.pack("<d", wall_time) + _len_field(3, b"brain.Event:2")


def frame_record(data: bytes) -> bytes:
    header = struct.pack("<Q", len(data))
    return header + struct.pack("<I", masked_crc32c(header)) + data + struct.pack("<I", masked_crc32c(data))


def read_records(path: str):
    """Parse a TFRecord file back into payloads (used by tests)."""
    out = []
    with open(path, "rb") as f:
        while True:
            h = f.read(8)
            if not h:
                break
            (n,) = struct.unpack("<Q", h)
            (hc,) = struct.unpack("<I", f.read(4))
            assert hc == masked_crc32c(h), "header crc mismatch"
            data = f.read(n)
            (dc,) = struct.unpack("<I", f.read(4))
            assert dc == masked_crc32c(data), "data crc mismatch"
            out.append(data)
    return out


class SummaryWriter:
    def __init__(self, logdir: str | None = None, comment: str = "", flush_secs: int = 10):
        if logdir is None:
            stamp = datetime.now().strftime("%b%d_%H-%M-%S")
            logdir = os.path.join("runs", f"{stamp}_{socket.gethostname()}{comment}")
        os.makedirs(logdir, exist_ok=True)
        self.logdir = logdir
        now = time.time()
        self._path = os.path.join(logdir, f"events.out.tfevents.{int(now)}.{socket.gethostname()}")
        self._f = open(self._path, "ab")
        self._jsonl = open(os.path.join(logdir, "scalars.jsonl"), "a")
        self._lock = threading.Lock()
        self._last_flush = now
        self._flush_secs = flush_secs
        self._f.write(frame_record(encode_version_event(now)))

    def add_scalar(self, tag, scalar_value, global_step=None, walltime=None):
        if hasattr(scalar_value, "item"):
            scalar_value = scalar_value.item()
        wt = time.time() if walltime is None else walltime
        step = 0 if global_step is None else int(global_step)
        rec = frame_record(encode_scalar_event(tag, float(scalar_value), step, wt))
        with self._lock:
            self._f.write(rec)
            self._jsonl.write(json.dumps({"tag": tag, "value": float(scalar_value), "step": step, "t": wt}) + "\n")
            if wt - self._last_flush > self._flush_secs:
                self.flush()

    def add_scalars(self, main_tag, tag_scalar_dict, global_step=None, walltime=None):
        for k, v in tag_scalar_dict.items():
            self.add_scalar(f"{main_tag}/{k}", v, global_step, walltime)

    def flush(self):
        self._f.flush()
        self._jsonl.flush()
        self._last_flush = time.time()

    def close(self):
        with self._lock:
            self.flush()
            self._f.close()
            self._jsonl.close()

    @property
    def event_path(self):
        return self._path


class NullWriter:
    """Drop-in writer that records nothing (benchmarks)."""

    def add_scalar(self, *a, **k):
        pass

    def add_scalars(self, *a, **k):
        pass

    def flush(self):
        pass

    def close(self):
        pass
