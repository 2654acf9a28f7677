"""Host replay: native segment trees / PER vs pure-Python oracles and the reference."""
import random

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from apex_amd.memory import (CustomPrioritizedReplayBuffer, CustomPrioritizedReplayBuffer_AQL,
                             PrioritizedReplayBuffer, ReplayBuffer)
from apex_amd.replay.segment_tree import MinSegmentTree, SegmentTree, SumSegmentTree

from . import refimport


def test_capacity_must_be_pow2():
    with pytest.raises(AssertionError):
        SumSegmentTree(6)
    with pytest.raises(AssertionError):
        SegmentTree(12, min, float("inf"))


@settings(max_examples=60, deadline=None)
@given(st.lists(st.tuples(st.integers(0, 31), st.floats(0.0, 100.0, allow_nan=False)), min_size=1, max_size=80),
       st.integers(0, 31), st.integers(1, 32))
def test_sum_min_tree_vs_python_oracle(writes, start, end):
    s, m = SumSegmentTree(32), MinSegmentTree(32)
    os_, om = SegmentTree(32, lambda a, b: a + b, 0.0), SegmentTree(32, min, float("inf"))
    for i, v in writes:
        s[i] = v
        m[i] = v
        os_[i] = v
        om[i] = v
    assert s.sum() == os_.reduce()
    assert m.min() == om.reduce()
    if start < end:
        assert s.sum(start, end) == os_.reduce(start, end)
        assert m.min(start, end) == om.reduce(start, end)
    total = s.sum()
    for frac in (0.0, 0.3, 0.77, 0.999):
        mass = frac * total
        # oracle descent
        idx = 1
        pm = mass
        while idx < 32:
            if os_._value[2 * idx] > pm:
                idx *= 2
            else:
                pm -= os_._value[2 * idx]
                idx = 2 * idx + 1
        assert s.find_prefixsum_idx(mass) == idx - 32


def test_batch_ops_last_write_wins():
    s = SumSegmentTree(16)
    s.set_batch([3, 5, 3], [1.0, 2.0, 7.0])
    assert s[3] == 7.0 and s.sum() == 9.0
    np.testing.assert_array_equal(s.find_prefixsum_idx_batch([0.0, 6.9, 7.0, 8.9]), [3, 3, 5, 5])


def test_uniform_replay_roundtrip():
    rb = ReplayBuffer(3)
    for i in range(5):
        rb.add(np.full(2, i), i, float(i), np.full(2, i + 1), False)
    assert len(rb) == 3
    random.seed(0)
    o, a, r, o2, d = rb.sample(10)
    assert o.shape == (10, 2) and set(a.tolist()) <= {2, 3, 4}


@pytest.mark.skipif(not refimport.available(), reason="reference not mounted")
@pytest.mark.parametrize("exact", [False])
def test_per_matches_reference_exactly(exact):
    ref = refimport.load("memory")
    ours = PrioritizedReplayBuffer(100, 0.6, exact_mass=exact)
    theirs = ref.PrioritizedReplayBuffer(100, 0.6)
    rng = np.random.RandomState(0)
    for i in range(150):
        tr = (rng.randn(3).astype(np.float32), i % 4, float(rng.randn()), rng.randn(3).astype(np.float32), i % 9 == 0)
        ours.add(*tr)
        theirs.add(*tr)
        if i > 40 and i % 10 == 0:
            random.seed(i)
            so = ours.sample(16, 0.4)
            random.seed(i)
            st_ = theirs.sample(16, 0.4)
            assert list(so[-1]) == list(st_[-1])
            np.testing.assert_allclose(so[-2], st_[-2], rtol=0, atol=0)
            for x, y in zip(so[:5], st_[:5]):
                np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
            pr = rng.uniform(0.1, 5, 16)
            ours.update_priorities(so[-1], pr)
            theirs.update_priorities(st_[-1], pr)
    assert ours._max_priority == theirs._max_priority
    assert ours._it_sum.sum() == theirs._it_sum.sum()
    assert ours._it_min.min() == theirs._it_min.min()


@pytest.mark.skipif(not refimport.available(), reason="reference not mounted")
def test_custom_per_matches_reference():
    ref = refimport.load("memory")
    ours = CustomPrioritizedReplayBuffer(64, 0.6)
    theirs = ref.CustomPrioritizedReplayBuffer(64, 0.6)
    rng = np.random.RandomState(1)
    for i in range(100):
        tr = (rng.randint(0, 255, (4, 2, 2)).astype(np.uint8), i % 6, float(rng.randn()),
              rng.randint(0, 255, (4, 2, 2)).astype(np.uint8), np.float32(i % 7 == 0), float(rng.uniform(0.01, 3)))
        ours.add(*tr)
        theirs.add(*tr)
    random.seed(5)
    a = ours.sample(32, 0.4)
    random.seed(5)
    b = theirs.sample(32, 0.4)
    assert isinstance(a[0], list) and isinstance(a[3], list)
    assert a[-1] == b[-1]
    np.testing.assert_array_equal(a[-2], b[-2])
    for x, y in zip(a[0], b[0]):
        np.testing.assert_array_equal(x, y)


def test_exact_mass_includes_newest_slot():
    """Q5: reference mass excludes slot len-1; exact_mass samples it."""
    ref_mode = PrioritizedReplayBuffer(8, 1.0, exact_mass=False)
    exact = PrioritizedReplayBuffer(8, 1.0, exact_mass=True)
    for buf in (ref_mode, exact):
        for i in range(4):
            buf.add(i, 0, 0.0, i, False)
        buf.update_priorities([0, 1, 2, 3], [1e-6, 1e-6, 1e-6, 100.0])
    random.seed(0)
    assert 3 not in ref_mode.sample(8, 0.4)[-1]
    random.seed(0)
    assert exact.sample(8, 0.4)[-1].count(3) >= 7


def test_aql_buffer_roundtrip():
    buf = CustomPrioritizedReplayBuffer_AQL(16, 0.6)
    for i in range(10):
        buf.add(np.ones(3) * i, i % 2, 1.0, np.ones(3), False, np.arange(5) + i)
    random.seed(2)
    s, a, r, s2, d, a_mu, w, idx = buf.sample(4, 0.4)
    assert a_mu.shape == (4, 5) and s.shape == (4, 3) and w.shape == (4,)
