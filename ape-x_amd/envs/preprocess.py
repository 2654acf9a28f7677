"""Atari preprocessing as one explicit pipeline.

The reference builds its observation pipeline by stacking a dozen gym wrappers
(origin_repo/wrapper.py:11-329, composed by ``make_atari`` / ``wrap_atari_dqn``).  Here the
pipeline is a single object, :class:`AtariPreprocess`, vectorised over N raw emulators and
configured by explicit flags (:class:`PreprocessSpec`): no-op randomised starts, action
repeat with a max over the last two frames, life-loss episode ends, the FIRE start
sequence, area resampling to 84x84 grey, reward sign clipping, frame stacking, float
scaling and the channels-first layout.  Every stage is a small function or class below;
the reference-named wrapper classes in :mod:`apex_amd.envs.atari` are thin adapters over
these same stages, so a user stacking ``wrap_atari_dqn(make_atari(id), args)`` and the
vector pipeline see identical streams (``tests/test_envs_host.py`` checks that).

Stage semantics (the reference's observable behaviour):

* **start** -- a real (game-over) start resets the emulator and plays ``U{1..noop_max}``
  raw NOOP frames (re-resetting if the game ends meanwhile); after a mere life loss the
  emulator is not reset, one repeated NOOP action is played instead.  Games with a FIRE
  action then play FIRE and action 2 (each through the life ledger; an episode end in
  between restarts), and the observation of the second is returned.
* **repeat** -- one agent step = ``skip`` emulator frames of the same action, rewards
  summed, observation = pixel-wise max of the last two frames *of this window*
  (the reference's fixed two-slot buffer can return frames of an earlier window when the
  game ends early in the window; here the pool only ever holds this window's frames).
* **life ledger** -- an agent-level episode ends when the lives counter drops (while
  lives remain); the emulator's own game-over is remembered for the next start.
* **warp** -- grey = 0.299 R + 0.587 G + 0.114 B, then separable area averaging
  (OpenCV INTER_AREA for downscaling) rounded to uint8.
* **layout** -- channels-first frames are ``swapaxes(2, 0)`` of the HWC frame, i.e.
  H and W are transposed (harmless at 84x84, kept so checkpoints see the same inputs);
  values stay 0..255 unless ``scale``.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

GREY = np.array([0.299, 0.587, 0.114])


# ---------------------------------------------------------------------------- stages
def meaning(env, index: int) -> str:
    return env.unwrapped.get_action_meanings()[index]


def has_fire(env) -> bool:
    return "FIRE" in env.unwrapped.get_action_meanings()


def lives_of(env) -> int:
    return int(env.unwrapped.ale.lives())


class RepeatPool:
    """Action repeat with a max-pool over two emulator frames.

    ``reference=True`` (default; origin_repo/wrapper.py:99-124 MaxAndSkipEnv): a PERSISTENT
    two-slot buffer written only at repeat steps ``repeat - 2`` and ``repeat - 1``, so when
    the episode ends earlier in the window the pooled frame still holds frames of an earlier
    window (the reference notes the done-frame observation "doesn't matter"; it is kept
    bit-exact here).  ``reference=False``: the max of the last two frames of THIS window
    (the done frame itself when the window ends after one step)."""

    def __init__(self, repeat: int = 4, reference: bool = True):
        self.repeat = int(repeat)
        self.reference = bool(reference)
        self._slots = None

    def reset(self) -> None:
        """Forget the persistent slots (a fresh emulator)."""
        self._slots = None

    def run(self, step_fn, action):
        total, prev, last, done, info = 0.0, None, None, False, {}
        for i in range(self.repeat):
            frame, r, done, info = step_fn(action)
            if self.reference:
                if self._slots is None:
                    f = np.asarray(frame)
                    self._slots = np.zeros((2,) + f.shape, dtype=f.dtype)
                if i == self.repeat - 2:
                    self._slots[0] = frame
                if i == self.repeat - 1:
                    self._slots[1] = frame
            prev, last = last, frame
            total += r
            if done:
                break
        if self.reference:
            return self._slots.max(axis=0), total, done, info
        pooled = last if prev is None else np.maximum(prev, last)
        return pooled, total, done, info


class LifeLedger:
    """Lives bookkeeping for life-loss episode ends.  ``game_over`` is the emulator's own
    terminal flag of the last step; ``observe`` turns a lost life into an agent-level end."""

    def __init__(self):
        self.lives = 0
        self.game_over = True

    def observe(self, done: bool, lives: int) -> bool:
        self.game_over = bool(done)
        lost = 0 < lives < self.lives
        self.lives = lives
        return bool(done) or lost


def noop_start(env, noop_max: int, fixed: int | None = None, reset_kwargs=None):
    """Emulator reset + ``fixed`` or U{1..noop_max} raw NOOP frames."""
    kw = reset_kwargs or {}
    obs = env.reset(**kw)
    n = fixed if fixed is not None else int(env.unwrapped.np_random.randint(1, noop_max + 1))
    if n <= 0:
        raise ValueError("the no-op start needs at least one NOOP frame")
    for _ in range(n):
        obs, _, done, _ = env.step(0)
        if done:
            obs = env.reset(**kw)
    return obs


def life_start(ledger: LifeLedger, hard_reset, soft_step, lives_fn):
    """Start of an agent-level episode: a real reset after a game over, otherwise one
    NOOP agent step (the game continues with a life fewer)."""
    obs = hard_reset() if ledger.game_over else soft_step(0)[0]
    ledger.lives = lives_fn()
    return obs


def fire_start(start, step):
    """FIRE, then action 2; an episode end after either restarts (the returned observation
    is the second step's, as in the reference)."""
    obs = start()
    for a in (1, 2):
        obs, _, done, _ = step(a)
        if done:
            start()
    return obs


def sign_reward(r) -> float:
    return float(np.sign(r))


def area_weights(n_out: int, n_in: int) -> np.ndarray:
    """[n_out, n_in] row-stochastic overlap weights of output pixel o = [o s, (o+1) s) in
    input pixels, s = n_in / n_out (area averaging, OpenCV INTER_AREA for downscale)."""
    s = n_in / n_out
    edges_lo = np.arange(n_out)[:, None] * s
    edges_hi = edges_lo + s
    pix = np.arange(n_in)[None, :]
    w = np.clip(np.minimum(edges_hi, pix + 1) - np.maximum(edges_lo, pix), 0.0, None)
    return w / w.sum(1, keepdims=True)


class AreaResize:
    """frame [H, W, 3] u8 -> [h, w, 1] grey (or [h, w, 3]) u8 by separable area averaging."""

    def __init__(self, in_hw, size=(84, 84), grayscale: bool = True):
        h, w = size
        self.out_hw = (h, w)
        self.grayscale = grayscale
        self.rows = area_weights(h, in_hw[0])
        self.cols = area_weights(w, in_hw[1]).T

    @property
    def channels(self) -> int:
        return 1 if self.grayscale else 3

    def __call__(self, frame: np.ndarray) -> np.ndarray:
        f = frame.astype(np.float64)
        if self.grayscale:
            out = (self.rows @ (f @ GREY) @ self.cols)[..., None]
        else:
            out = np.einsum("hi,iwc->hwc", self.rows, np.einsum("iwc,wv->ivc", f, self.cols))
        return np.clip(np.rint(out), 0, 255).astype(np.uint8)


def channels_first(frame: np.ndarray) -> np.ndarray:
    """HWC -> C,W,H via swapaxes(2, 0) (H/W transposed)."""
    return np.swapaxes(frame, 2, 0)


# ---------------------------------------------------------------------------- pipeline
@dataclass(frozen=True)
class PreprocessSpec:
    noop_max: int = 30
    skip: int = 4
    episode_life: bool = True
    fire_reset: bool | None = None     # None: iff the game has a FIRE action
    size: tuple = (84, 84)
    grayscale: bool = True
    clip_rewards: bool = True
    stack: int = 4                     # 0 / 1: no stacking
    scale: bool = False
    channels_first: bool = True        # ImageToPyTorch layout (the Ape-X actor's)
    reference_pool: bool = True        # MaxAndSkipEnv's persistent two-slot buffer (RepeatPool)

    @classmethod
    def from_args(cls, args) -> "PreprocessSpec":
        """The reference's env flags (arguments.py:19-27: episode_life, clip_rewards,
        frame_stack, scale)."""
        return cls(episode_life=bool(args.episode_life), clip_rewards=bool(args.clip_rewards),
                   stack=4 if args.frame_stack else 1, scale=bool(args.scale))


class AtariPreprocess:
    """The whole preprocessing pipeline over N raw emulators (each ``make(id)``-style:
    ``get_action_meanings``, ``ale.lives()``, ``np_random``).

    ``reset()`` starts every env and returns obs ``[N, ...]``; ``reset_one(i)`` restarts
    env i; ``step(actions)`` returns ``(obs [N, ...], reward [N], done [N], infos)`` with the
    agent-level done (life loss included when ``episode_life``).  Observations are
    ``[k, h, w]`` (channels-first, H/W transposed) or ``[h, w, k]``, uint8 0..255, or
    float32 /255 with ``scale``.  Envs are not auto-reset: restart them with ``reset_one``.
    The envs are stepped one after another (a Python loop over emulators: each step is an
    emulator call plus numpy resize / stack work); only the frame stacks are one array.
    """

    def __init__(self, raw_envs, spec: PreprocessSpec = PreprocessSpec()):
        self.envs = list(raw_envs)
        self.spec = spec
        self.fixed_noops: list[int | None] = [None] * len(self.envs)
        e0 = self.envs[0]
        if meaning(e0, 0) != "NOOP":
            raise ValueError("action 0 must be NOOP")
        fire = has_fire(e0) if spec.fire_reset is None else spec.fire_reset
        if fire and (meaning(e0, 1) != "FIRE" or len(e0.unwrapped.get_action_meanings()) < 3):
            raise ValueError("the FIRE start needs FIRE at action 1 and at least 3 actions")
        self.fire = fire
        self.pools = [RepeatPool(spec.skip, spec.reference_pool) for _ in self.envs]  # per-env slots
        self.ledgers = [LifeLedger() for _ in self.envs]
        self.resize = AreaResize(e0.observation_space.shape[:2], spec.size, spec.grayscale)
        h, w = spec.size
        c = self.resize.channels
        self.k = max(1, int(spec.stack))
        frame_shape = (c, w, h) if spec.channels_first else (h, w, c)
        self.cat_axis = 0 if spec.channels_first else 2
        self.frame_shape = frame_shape
        stacked = list(frame_shape)
        stacked[self.cat_axis] *= self.k
        self.obs_shape = tuple(stacked)
        self._frames = np.zeros((len(self.envs), self.k) + frame_shape, dtype=np.uint8)
        self.action_space = e0.action_space
        self.observation_space_shape = self.obs_shape

    def __len__(self) -> int:
        return len(self.envs)

    # -- per-env stages composed in the reference order
    def _repeat(self, i, a):
        return self.pools[i].run(self.envs[i].step, a)

    def _agent_step(self, i, a):
        frame, r, done, info = self._repeat(i, a)
        if self.spec.episode_life:
            done = self.ledgers[i].observe(done, lives_of(self.envs[i]))
        return frame, r, done, info

    def _hard_start(self, i):
        return noop_start(self.envs[i], self.spec.noop_max, self.fixed_noops[i])

    def _start(self, i):
        if self.spec.episode_life:
            return life_start(self.ledgers[i], lambda: self._hard_start(i), lambda a: self._repeat(i, a),
                              lambda: lives_of(self.envs[i]))
        return self._hard_start(i)

    def _frame(self, raw):
        f = self.resize(raw)
        return channels_first(f) if self.spec.channels_first else f

    def _emit(self, i):
        obs = np.concatenate(list(self._frames[i]), axis=self.cat_axis)
        return obs.astype(np.float32) / 255.0 if self.spec.scale else obs

    def reset_one(self, i: int):
        raw = fire_start(lambda: self._start(i), lambda a: self._agent_step(i, a)) if self.fire else self._start(i)
        self._frames[i] = self._frame(raw)   # the start frame fills the whole stack
        return self._emit(i)

    def reset(self):
        return np.stack([self.reset_one(i) for i in range(len(self.envs))])

    def step(self, actions):
        n = len(self.envs)
        obs, rew = [], np.zeros(n, dtype=np.float64)
        done = np.zeros(n, dtype=bool)
        infos = []
        for i in range(n):
            raw, r, d, info = self._agent_step(i, int(actions[i]))
            self._frames[i, :-1] = self._frames[i, 1:]
            self._frames[i, -1] = self._frame(raw)
            rew[i] = sign_reward(r) if self.spec.clip_rewards else r
            done[i] = d
            infos.append(info)
            obs.append(self._emit(i))
        return np.stack(obs), rew, done, infos

    def seed(self, seed: int) -> None:
        for i, e in enumerate(self.envs):
            e.seed(seed + i)
