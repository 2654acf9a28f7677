"""Host n-step batcher: reference-mode parity (Q1-Q4) and textbook semantics."""
import numpy as np
import pytest

from apex_amd.replay.nstep import BatchStorage

from . import refimport


def _drive(bs, rewards, dones, A=3, seed=0):
    rng = np.random.RandomState(seed)
    for t, (r, d) in enumerate(zip(rewards, dones)):
        bs.add(f"s{t}", r, t % A, d, rng.randn(A).astype(np.float32))
    return bs


def test_q1_reference_sums_n_plus_one_rewards():
    bs = _drive(BatchStorage(3, 0.5), [1, 2, 3, 4, 5, 6], [0, 0, 0, 0, 0, 0])
    # R(s0) = 1 + .5*2 + .25*3 + .125*4 = 3.25 with next = s3
    assert bs.states[0] == "s0" and bs.next_states[0] == "s3"
    assert bs.rewards[0] == pytest.approx(1 + 1 + 0.75 + 0.5)


def test_q2_q4_done_semantics():
    bs = _drive(BatchStorage(3, 0.5), [1, 1, 1, 1, 1, 1], [0, 0, 0, 0, 0, 1])
    assert bs.states == ["s0", "s1", "s2"]  # tail s3, s4 dropped on done
    assert bs.next_states[-1] == "s5" and bs.dones[-1] == 1.0
    bs2 = _drive(BatchStorage(3, 0.5), [1], [1])  # Q4: no IndexError
    assert len(bs2) == 0


def test_textbook_mode():
    bs = _drive(BatchStorage(3, 0.5, mode="textbook"), [1, 2, 3, 4, 5], [0, 0, 0, 0, 1])
    assert bs.states == ["s0", "s1", "s2", "s3", "s4"]
    assert bs.next_states[0] == "s3" and bs.dones[0] == 0.0
    assert bs.rewards[0] == pytest.approx(1 + 0.5 * 2 + 0.25 * 3)
    assert bs.dones[2:] == [1.0, 1.0, 1.0]
    assert bs.rewards[4] == pytest.approx(5.0)
    assert bs.rewards[3] == pytest.approx(4 + 0.5 * 5)
    pr = bs.compute_priorities()
    assert pr.shape == (5,) and (pr > 0).all()


@pytest.mark.skipif(not refimport.available(), reason="reference not mounted")
def test_reference_mode_matches_reference_batchstorage():
    ref = refimport.load("memory")
    rng = np.random.RandomState(3)
    T, A = 400, 6
    rewards = rng.randn(T)
    dones = rng.rand(T) < 0.06
    dones[0] = False
    ours, theirs = BatchStorage(3, 0.99), ref.BatchStorage(3, 0.99)
    qs = rng.randn(T, A).astype(np.float32)
    for t in range(T):
        args = (rng.randn(2).astype(np.float32), float(rewards[t]), int(t % A), bool(dones[t]), qs[t])
        if dones[t] and len(theirs.state_deque) == 0:
            # the reference raises IndexError here (Q4); ours emits nothing
            with pytest.raises(IndexError):
                theirs.add(*args)
            ours.add(*args)
            continue
        ours.add(*args)
        theirs.add(*args)
        if len(theirs) >= 50:
            (b1, p1), (b2, p2) = ours.make_batch(), theirs.make_batch()
            np.testing.assert_allclose(p1, p2, rtol=1e-12)
            for x, y in zip(b1, b2):
                np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
            ours.reset()
            theirs.reset()
