"""Segment trees (reference memory.py:10-143).

``SegmentTree`` keeps the reference's generic signature (any associative
``operation`` + ``neutral_element``) as a pure-Python array tree.
``SumSegmentTree`` / ``MinSegmentTree`` -- the two the replay actually uses -- are
backed by the native C++ ``_apex_cpu.Tree`` (flat double arrays, same recursion and
combine order, so results are bitwise equal to the reference).

Semantics kept: capacity must be a power of two; ``reduce(start, end)`` treats
``end`` as exclusive (``None`` = capacity, negative wraps); ``find_prefixsum_idx``
asserts ``0 <= mass <= sum() + 1e-5``.
"""
from __future__ import annotations

import numpy as np

from .. import ops


class SegmentTree:
    def __init__(self, capacity, operation, neutral_element):
        assert capacity > 0 and capacity & (capacity - 1) == 0, "capacity must be positive and a power of 2."
        self._capacity = int(capacity)
        self._value = [neutral_element] * (2 * self._capacity)
        self._operation = operation
        self._neutral = neutral_element

    def _reduce_helper(self, start, end, node, node_start, node_end):
        # iterative-free recursion identical in combine order to the reference
        if start == node_start and end == node_end:
            return self._value[node]
        mid = (node_start + node_end) // 2
        if end <= mid:
            return self._reduce_helper(start, end, 2 * node, node_start, mid)
        if mid + 1 <= start:
            return self._reduce_helper(start, end, 2 * node + 1, mid + 1, node_end)
        return self._operation(self._reduce_helper(start, mid, 2 * node, node_start, mid),
                               self._reduce_helper(mid + 1, end, 2 * node + 1, mid + 1, node_end))

    def reduce(self, start=0, end=None):
        if end is None:
            end = self._capacity
        if end < 0:
            end += self._capacity
        end -= 1
        if end < start:
            return self._neutral
        return self._reduce_helper(start, end, 1, 0, self._capacity - 1)

    def __setitem__(self, idx, val):
        i = int(idx) + self._capacity
        self._value[i] = val
        i //= 2
        while i >= 1:
            self._value[i] = self._operation(self._value[2 * i], self._value[2 * i + 1])
            i //= 2

    def __getitem__(self, idx):
        assert 0 <= idx < self._capacity
        return self._value[self._capacity + idx]


class _NativeTree:
    _op = "sum"

    def __init__(self, capacity):
        assert capacity > 0 and capacity & (capacity - 1) == 0, "capacity must be positive and a power of 2."
        self._capacity = int(capacity)
        self._t = ops.cpu().Tree(self._capacity, self._op)

    @classmethod
    def _wrap(cls, native_tree):
        obj = cls.__new__(cls)
        obj._capacity = native_tree.capacity
        obj._t = native_tree
        return obj

    def reduce(self, start=0, end=None):
        return self._t.reduce(int(start), None if end is None else int(end))

    def __setitem__(self, idx, val):
        self._t.set(int(idx), float(val))

    def __getitem__(self, idx):
        assert 0 <= idx < self._capacity
        return self._t.get(int(idx))

    def set_batch(self, idxes, values):
        self._t.set_batch(np.asarray(idxes, dtype=np.int64), np.asarray(values, dtype=np.float64))

    @property
    def _value(self):
        return self._t.values().tolist()


class SumSegmentTree(_NativeTree):
    _op = "sum"

    def sum(self, start=0, end=None):
        return self.reduce(start, end)

    def find_prefixsum_idx(self, prefixsum):
        assert 0 <= prefixsum <= self.sum() + 1e-5
        return int(self._t.find_prefixsum_idx(float(prefixsum)))

    def find_prefixsum_idx_batch(self, masses):
        return self._t.find_prefixsum_idx_batch(np.asarray(masses, dtype=np.float64))


class MinSegmentTree(_NativeTree):
    _op = "min"

    def min(self, start=0, end=None):
        return self.reduce(start, end)
