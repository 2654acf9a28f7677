"""Single-node actor workers (reference batchrecorder.py:13-152, batchrecoder_AQL.py:13-138;
SURVEY R7, R8, M8).

Same role as the reference ``BatchRecorder``: ``n_workers`` CPU processes, each with
its own env, a CPU copy of the policy and (DQN) a :class:`BatchStorage` n-step
batcher, with the Ape-X epsilon ladder ``eps_i = 0.4^(1 + 7 i/(N-1))``.

Differences by design (documented fixes):

* **Addressed tasks** -- one task queue per worker, so every worker gets every
  weight update and exactly one ``record_batch`` (the reference shares a
  JoinableQueue).
* **Weights via shared memory** -- :class:`~apex_amd.parallel.shm.SharedParams`
  (one flat buffer + seqlock version) instead of pickling the state_dict once per
  worker per publish.
* **Continuous mode** -- ``start()`` lets workers play episodes back to back and
  stream chunks of ``send_interval`` transitions through a bounded result queue
  (credit-style back-pressure like origin ``max_outstanding``), so the learner trains
  concurrently with acting (the reference's ``ApeX.py`` collects only once, Q7).
  ``record_batch()`` keeps the reference one-episode-per-worker round.
* A crashed worker is detected (``is_alive``) instead of hanging ``join()``.

``BatchRecorder.record_batch()`` returns the number of transitions inserted (DQN) or
the total episode length (AQL, like batchrecoder_AQL.py:110-123).  The AQL duplicate
insertion quirk (each transition inserted ``len(state)`` times) is
available as ``aql_dup_by_obs_dim=True`` (default off).
"""
from __future__ import annotations

import multiprocessing as mp
import queue as _queue
import random
import time

import numpy as np
import torch

from ..algo.schedules import actor_epsilon
from ..parallel.shm import SharedParams

KIND_DQN = "dqn"
KIND_AQL = "aql"


def _seed_all(seed: int) -> None:
    np.random.seed(seed)
    random.seed(seed)
    torch.manual_seed(seed)


class Worker(mp.Process):
    """One actor process.  Built lazily in ``run`` so it works with ``spawn``."""

    def __init__(self, worker_id, env_id, seed, epsilon, task_queue, result_queue, params: SharedParams,
                 max_episode_length=50000, kind=KIND_DQN, n_steps=3, gamma=0.99, send_interval=50,
                 nstep_mode="reference", update_interval=400, aql_kwargs=None, stop_event=None):
        super().__init__(daemon=True)
        self.worker_id = int(worker_id)
        self.env_id = env_id
        self.seed = int(seed)
        self.epsilon = float(epsilon)
        self.task_queue = task_queue
        self.result_queue = result_queue
        self.params = params
        self.max_episode_length = int(max_episode_length)
        self.kind = kind
        self.n_steps, self.gamma = int(n_steps), float(gamma)
        self.send_interval = int(send_interval)
        self.nstep_mode = nstep_mode
        self.update_interval = int(update_interval)
        self.aql_kwargs = dict(aql_kwargs or {})
        self.stop_event = stop_event

    # ------------------------------------------------------------------ setup
    def _build(self):
        from .. import envs

        torch.set_num_threads(1)
        self.env = envs.make(self.env_id)
        self.env.seed(self.seed)
        _seed_all(self.seed)
        if self.kind == KIND_DQN:
            from ..models.dqn import DuelingDQN
            from ..replay.nstep import BatchStorage

            self.model = DuelingDQN(self.env)
            self.storage = BatchStorage(self.n_steps, self.gamma, mode=self.nstep_mode)
        else:
            from ..models.aql import AQL

            self.model = AQL(self.env, device="cpu", **self.aql_kwargs)
        self.version = 0
        self.steps = 0

    def _pull(self):
        self.version = self.params.pull(self.model, self.version)

    # ------------------------------------------------------------------ episodes
    def _dqn_episode(self):
        """One episode (batchrecorder.py:42-78): chunks of ``send_interval`` stored
        transitions (or the tail at ``done``) go to the result queue."""
        ep_r, ep_len = 0.0, 0
        state = self.env.reset()
        self.storage.reset()
        while True:
            action, q = self.model.act(torch.as_tensor(np.asarray(state), dtype=torch.float32), self.epsilon)
            next_state, reward, done, _ = self.env.step(action)
            self.storage.add(state, reward, action, done, q)
            state = next_state
            ep_r += reward
            ep_len += 1
            self.steps += 1
            if self.steps % self.update_interval == 0:
                self._pull()
                if self.stop_event is not None and self.stop_event.is_set():
                    return  # continuous mode is stopping: drop the partial window
            if done or ep_len >= self.max_episode_length:
                self.result_queue.put(("episode", self.worker_id, float(ep_r), int(ep_len)))
                if not done:  # truncated: the reference resets and keeps playing
                    state = self.env.reset()
                    ep_r, ep_len = 0.0, 0
            if done or len(self.storage) >= self.send_interval:
                batch, prios = self.storage.make_batch()
                if len(prios):
                    self.result_queue.put(("chunk", self.worker_id, (*batch, prios)))
                self.storage.reset()
            if done:
                return

    def _aql_episode(self):
        """One raw-transition episode with candidate sets (batchrecoder_AQL.py:38-59)."""
        ep_r, ep_len = 0.0, 0
        state = self.env.reset()
        memory = []
        while True:
            action, a_mu, _ = self.model.act(state, self.epsilon)
            a_mu = a_mu[0]
            next_state, reward, done, _ = self.env.step(a_mu[action])
            memory.append((state, action, reward, next_state, done, a_mu))
            state = next_state
            ep_r += reward
            ep_len += 1
            self.steps += 1
            if done or ep_len >= self.max_episode_length:
                break
        self.result_queue.put(("aql", self.worker_id, memory, float(ep_r), int(ep_len)))

    def _episode(self):
        (self._dqn_episode if self.kind == KIND_DQN else self._aql_episode)()

    # ------------------------------------------------------------------ task loop
    def run(self):
        self._build()
        while True:
            task = self.task_queue.get()
            desc = task["desc"]
            if desc == "record_batch":
                self._pull()
                self._episode()
                self.result_queue.put(("done", self.worker_id))
            elif desc == "set_pi_weights":
                self._pull()
                self.result_queue.put(("ack", self.worker_id, self.version))
            elif desc == "run":
                self._pull()
                while not self.stop_event.is_set():
                    self._episode()
                    self._pull()
                self.result_queue.put(("done", self.worker_id))
            elif desc == "cleanup":
                self.env.close()
                self.result_queue.put(("bye", self.worker_id))
                return


class BatchRecorder:
    def __init__(self, env_id, env_seed, n_workers, buffer, n_steps=3, gamma=0.99, max_episode_length=50000,
                 send_interval=50, kind=KIND_DQN, writer=None, nstep_mode="reference", update_interval=400,
                 eps_base=0.4, eps_alpha=7.0, start_method="spawn", result_queue_size=64, aql_kwargs=None,
                 aql_dup_by_obs_dim=False, model=None):
        self.env_id = env_id
        self.n_workers = int(n_workers)
        self.buffer = buffer
        self.writer = writer
        self.kind = kind
        self.aql_dup_by_obs_dim = aql_dup_by_obs_dim
        self.episode_idx = 0
        self.episodes: list[tuple[float, int]] = []
        self.inserted = 0
        ctx = mp.get_context(start_method)
        self.ctx = ctx
        if model is None:
            from .. import envs

            env = envs.make(env_id)
            if kind == KIND_DQN:
                from ..models.dqn import DuelingDQN

                model = DuelingDQN(env)
            else:
                from ..models.aql import AQL

                model = AQL(env, device="cpu", **(aql_kwargs or {}))
            env.close()
        self.params = SharedParams.for_module(model, ctx)
        self.params.publish(model)
        self.result_queue = ctx.Queue(maxsize=result_queue_size)
        self.stop_event = ctx.Event()
        self.task_queues = [ctx.Queue() for _ in range(self.n_workers)]
        eps = actor_epsilon(np.arange(self.n_workers), self.n_workers, eps_base, eps_alpha)
        self.workers = [
            Worker(i, env_id, env_seed + i, float(np.atleast_1d(eps)[i]), self.task_queues[i], self.result_queue,
                   self.params, max_episode_length, kind, n_steps, gamma, send_interval, nstep_mode,
                   update_interval, aql_kwargs, self.stop_event)
            for i in range(self.n_workers)
        ]
        for w in self.workers:
            w.start()
        self.running = False

    # ------------------------------------------------------------------ results
    def _check_alive(self):
        dead = [w.worker_id for w in self.workers if not w.is_alive()]
        if dead:
            raise RuntimeError(f"actor workers {dead} died")

    def _get(self, timeout=1.0):
        while True:
            try:
                return self.result_queue.get(timeout=timeout)
            except _queue.Empty:
                self._check_alive()

    def _handle(self, msg) -> int:
        """Insert a worker message into the buffer; returns transitions inserted."""
        tag = msg[0]
        if tag == "chunk":
            states, actions, rewards, next_states, dones, prios = msg[2]
            self.buffer.add_batch(states, actions, rewards, next_states, dones, prios)
            self.inserted += len(prios)
            return len(prios)
        if tag == "episode":
            _, wid, ep_r, ep_len = msg
            self._log_episode(ep_r, ep_len)
            return 0
        if tag == "aql":
            _, wid, memory, ep_r, ep_len = msg
            self._log_episode(ep_r, ep_len)
            n = 0
            for (s, a, r, s2, d, a_mu) in memory:
                reps = len(s) if self.aql_dup_by_obs_dim else 1
                for _ in range(reps):
                    self.buffer.add(s, a, r, s2, d, a_mu)
                    n += 1
            self.inserted += n
            return n
        return 0

    def _log_episode(self, ep_r, ep_len):
        self.episodes.append((ep_r, ep_len))
        if self.writer is not None:
            self.writer.add_scalar("actor/episode_reward", ep_r, self.episode_idx)
            self.writer.add_scalar("actor/episode_length", ep_len, self.episode_idx)
        self.episode_idx += 1

    # ------------------------------------------------------------------ reference API
    def record_batch(self) -> int:
        """Every worker plays exactly one episode; everything is inserted before return.
        Returns transitions inserted (DQN) / total episode length (AQL)."""
        if self.running:
            raise RuntimeError("record_batch() while workers run continuously")
        for q in self.task_queues:
            q.put({"desc": "record_batch"})
        done, total_len, ep0 = 0, 0, len(self.episodes)
        while done < self.n_workers:
            msg = self._get()
            if msg[0] == "done":
                done += 1
            else:
                self._handle(msg)
        total_len = sum(l for _, l in self.episodes[ep0:])
        return total_len

    def set_worker_weights(self, model) -> int:
        """Publish ``model``'s weights (shared memory) and have every worker load them."""
        v = self.params.publish(model)
        if not self.running:
            for q in self.task_queues:
                q.put({"desc": "set_pi_weights"})
            acks = 0
            while acks < self.n_workers:
                msg = self._get()
                if msg[0] == "ack":
                    acks += 1
                else:
                    self._handle(msg)
        return v

    # ------------------------------------------------------------------ continuous mode
    def start(self) -> None:
        """Workers play episodes back to back until :meth:`stop`; weights are picked up
        every ``update_interval`` steps and at every episode boundary."""
        self.stop_event.clear()
        for q in self.task_queues:
            q.put({"desc": "run"})
        self.running = True

    def poll(self, max_msgs: int = 64, timeout: float = 0.0) -> int:
        """Drain up to ``max_msgs`` worker messages into the buffer (non-blocking by
        default); returns transitions inserted."""
        n = 0
        for i in range(max_msgs):
            try:
                msg = self.result_queue.get(timeout=timeout) if (timeout and i == 0) else \
                    self.result_queue.get_nowait()
            except _queue.Empty:
                self._check_alive()
                break
            n += self._handle(msg)
        return n

    def wait_for(self, n_transitions: int, timeout: float = 600.0) -> int:
        """Block until at least ``n_transitions`` have been inserted in total."""
        t0 = time.time()
        while self.inserted < n_transitions:
            if time.time() - t0 > timeout:
                raise TimeoutError(f"only {self.inserted}/{n_transitions} transitions after {timeout}s")
            self._handle(self._get())
        return self.inserted

    def stop(self) -> None:
        if not self.running:
            return
        self.stop_event.set()
        done = 0
        while done < self.n_workers:
            msg = self._get()
            if msg[0] == "done":
                done += 1
            else:
                self._handle(msg)
        self.running = False

    def cleanup(self) -> None:
        try:
            self.stop()
            for q in self.task_queues:
                q.put({"desc": "cleanup"})
            deadline = time.time() + 10
            for w in self.workers:
                w.join(timeout=max(0.1, deadline - time.time()))
        finally:
            for w in self.workers:
                if w.is_alive():
                    w.terminate()
                    w.join(timeout=5)
