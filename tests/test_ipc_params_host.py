"""The pinned parameter-publish protocol of parallel/ipc.py on the host: the writer's
version choice (pick_version) and the reader's pull (pinned_pull) over a real /dev/shm
ControlBlock, with the GPU copies modelled by host copies.  A reader whose pull is
arbitrarily slow still installs a clean version on its first try while the writer
publishes as fast as it can (the 2 ms conflation floor is gone)."""
import os
import threading
import time

import numpy as np

from apex_amd.parallel.ipc import ControlBlock, param_buffers, pick_version, pinned_pull


def test_pick_version_avoids_pinned_and_newest_buffers():
    K = param_buffers(3)
    assert K == 5
    assert pick_version(0, [0, 0, 0], K) == 1
    assert pick_version(4, [0, 0, 0], K) == 5          # buffer 0 (version 5) free
    assert pick_version(9, [5, 0, 0], K) == 11          # version 5 pinned (buffer 0 = version 10s) -> 11
    # every reader pinned on a different buffer + the newest: still a free one within K tries
    for last in range(20):
        for pins in ([last - 1, last - 2, last - 3], [last, last, last], [1, 2, 3]):
            v = pick_version(last, pins, K)
            assert v > last and v % K not in {p % K for p in pins if p > 0} | {last % K} and v - last <= K


def test_slow_reader_never_starves_while_writer_publishes_nonstop():
    R, P = 3, 4096
    name = f"apex_test_pin_{os.getpid()}"
    ctrl = ControlBlock(name, R, create=True)
    try:
        K = ctrl.K
        bufs = np.zeros((K, P), dtype=np.int64)
        stop = threading.Event()
        published = [0]

        def writer():  # the learner publishing every iteration (no clock floor)
            last = 0
            while not stop.is_set():
                v = pick_version(last, ctrl.view("pin"), K)
                b = v % K
                ctrl.w[ctrl.begin_off(b)] = v      # begin word, stream-ordered before the copy
                bufs[b, :] = v                      # the copy
                ctrl.w[2] = v                       # release the version
                last = v
                published[0] += 1

        th = threading.Thread(target=writer)
        th.start()
        try:
            out = np.zeros(P, dtype=np.int64)
            have, installs, fails = 0, 0, 0

            def slow_pull(b):  # a reader whose copy sits behind queued work: ~2 ms, element-wise chunks
                for j in range(0, P, 512):
                    out[j:j + 512] = bufs[b, j:j + 512]
                    time.sleep(0.00025)

            t_end = time.monotonic() + 2.0
            while time.monotonic() < t_end:
                v, failed = pinned_pull(ctrl, 1, have, slow_pull)
                fails += failed
                if v is None:
                    continue
                assert v > have and (out == v).all(), "torn or stale parameter pull"
                have, installs = v, installs + 1
            assert installs >= 50 and published[0] > 20 * installs  # the writer ran far ahead of the reader
            assert fails <= 2, fails  # a pull fails only if K versions land between reading the word and pinning
            assert ctrl.view("pin")[1] == 0  # unpinned between pulls
        finally:
            stop.set()
            th.join(10)
    finally:
        ctrl.unlink()
