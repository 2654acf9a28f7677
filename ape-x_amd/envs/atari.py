"""Atari-shaped environments and the DeepMind wrapper stack.

ALE / gym[atari] / OpenCV are not installed, so ``make_atari`` builds a seeded
*synthetic Atari emulator* with the same observable contract as an ALE
``*NoFrameskip-v4`` env: 210x160x3 uint8 RGB frames, the ALE action-meaning lists,
``ale.lives()``, ``np_random`` and raw (unclipped) game scores.  Preprocessing is the
pipeline of :mod:`apex_amd.envs.preprocess` (``AtariPreprocess``, vectorised, explicit
flags); the reference's wrapper names (origin_repo/wrapper.py: NoopReset, FireReset,
EpisodicLife, MaxAndSkip, ClipReward, WarpFrame, FrameStack/TorchFrameStack + LazyFrames,
ScaledFloatFrame, ImageToPyTorch, make_atari, wrap_deepmind, wrap_atari_dqn) are kept as
thin adapters over its stages.

The GPU-resident vector env used by the high-throughput engine
(`vec_env_step_k`, ops/csrc/actor_kernels.hip, driven by :mod:`apex_amd.engine.actor_shard`) renders the same game family straight to 84x84.
"""
from __future__ import annotations

from collections import deque

import numpy as np

from . import preprocess as P
from .core import Env, ObservationWrapper, RewardWrapper, TimeLimit, Wrapper, register
from .spaces import Box, Discrete

FULL_ACTIONS = ["NOOP", "FIRE", "UP", "RIGHT", "LEFT", "DOWN", "UPRIGHT", "UPLEFT", "DOWNRIGHT",
                "DOWNLEFT", "UPFIRE", "RIGHTFIRE", "LEFTFIRE", "DOWNFIRE", "UPRIGHTFIRE",
                "UPLEFTFIRE", "DOWNRIGHTFIRE", "DOWNLEFTFIRE"]
GAME_ACTIONS = {
    "Pong": ["NOOP", "FIRE", "RIGHT", "LEFT", "RIGHTFIRE", "LEFTFIRE"],
    "Breakout": ["NOOP", "FIRE", "RIGHT", "LEFT"],
    "Seaquest": FULL_ACTIONS,
    "SpaceInvaders": ["NOOP", "FIRE", "RIGHT", "LEFT", "RIGHTFIRE", "LEFTFIRE"],
    "MsPacman": ["NOOP", "UP", "RIGHT", "LEFT", "DOWN", "UPRIGHT", "UPLEFT", "DOWNRIGHT", "DOWNLEFT"],
}
GAME_LIVES = {"Pong": 0, "Breakout": 5, "Seaquest": 4, "SpaceInvaders": 3, "MsPacman": 3}


def is_atari_id(env_id: str) -> bool:
    return any(env_id.startswith(g) for g in GAME_ACTIONS) and ("NoFrameskip" in env_id or env_id.endswith("-v4")
                                                              or env_id.endswith("-v0"))


def game_of(env_id: str) -> str:
    for g in GAME_ACTIONS:
        if env_id.startswith(g):
            return g
    raise KeyError(env_id)


def action_delta(meaning: str) -> tuple[int, int, bool]:
    dx = (1 if "RIGHT" in meaning else 0) - (1 if "LEFT" in meaning else 0)
    dy = (1 if "DOWN" in meaning else 0) - (1 if "UP" in meaning else 0)
    return dx, dy, "FIRE" in meaning


class _ALEStub:
    def __init__(self, env):
        self._env = env

    def lives(self):
        return self._env.lives


class SyntheticAtariEnv(Env):
    """Deterministic (given the seed) sprite game with ALE's observable interface.

    Player ship moves with the action's direction, FIRE launches a projectile upward;
    enemies sweep horizontally and descend; hitting an enemy scores, touching one
    costs a life.  Frame = 210x160x3 uint8.  One ``step`` = one emulator frame
    (NoFrameskip), so MaxAndSkipEnv(4) gives the usual 4-frame action repeat.
    """

    H, W = 210, 160
    N_ENEMIES = 6

    def __init__(self, game: str = "Seaquest"):
        super().__init__()
        self.game = game
        self._meanings = list(GAME_ACTIONS[game])
        self.action_space = Discrete(len(self._meanings))
        self.observation_space = Box(0, 255, shape=(self.H, self.W, 3), dtype=np.uint8)
        self.ale = _ALEStub(self)
        self.lives = GAME_LIVES[game]
        self._frame = np.zeros((self.H, self.W, 3), dtype=np.uint8)
        self.reset()

    def get_action_meanings(self):
        return list(self._meanings)

    def reset(self):
        rng = self.np_random
        self.lives = GAME_LIVES[self.game]
        self.px, self.py = 76.0, 180.0
        self.ex = rng.uniform(8, self.W - 16, self.N_ENEMIES)
        self.ey = 20.0 + 18.0 * np.arange(self.N_ENEMIES)
        self.evx = rng.choice([-1.5, 1.5], self.N_ENEMIES) * rng.uniform(0.5, 1.5, self.N_ENEMIES)
        self.bullet = None
        self.t = 0
        self.score_since_point = 0
        return self._render()

    def step(self, action):
        dx, dy, fire = action_delta(self._meanings[int(action)])
        self.t += 1
        self.px = float(np.clip(self.px + 2.0 * dx, 0, self.W - 8))
        self.py = float(np.clip(self.py + 2.0 * dy, 100, self.H - 12))
        if fire and self.bullet is None:
            self.bullet = [self.px + 3.0, self.py - 4.0]
        reward = 0.0
        self.ex += self.evx
        bounce = (self.ex < 0) | (self.ex > self.W - 12)
        self.evx[bounce] *= -1.0
        self.ex = np.clip(self.ex, 0, self.W - 12)
        if self.t % 64 == 0:
            self.ey += 4.0
        if self.bullet is not None:
            self.bullet[1] -= 6.0
            hit = (np.abs(self.ex + 6 - self.bullet[0]) < 8) & (np.abs(self.ey + 4 - self.bullet[1]) < 6)
            if hit.any():
                k = int(np.argmax(hit))
                reward += 20.0 if self.game == "Seaquest" else 1.0
                self.ex[k] = self.np_random.uniform(8, self.W - 16)
                self.ey[k] = 20.0
                self.bullet = None
            elif self.bullet[1] < 0:
                self.bullet = None
        done = False
        crash = (np.abs(self.ex + 6 - (self.px + 4)) < 9) & (np.abs(self.ey + 4 - (self.py + 4)) < 8)
        if crash.any() or (self.ey > self.H - 20).any():
            if self.game == "Pong":
                reward -= 1.0
                self.ey[:] = 20.0 + 18.0 * np.arange(self.N_ENEMIES)
                self.score_since_point += 1
                done = self.score_since_point >= 21
            else:
                self.lives -= 1
                self.ey[:] = 20.0 + 18.0 * np.arange(self.N_ENEMIES)
                done = self.lives <= 0
        return self._render(), reward, done, {"ale.lives": self.lives}

    def _render(self):
        f = self._frame
        f[:] = (0, 28, 136)
        f[:12] = (24, 26, 167)
        f[self.H - 10:] = (142, 142, 142)
        x, y = int(self.px), int(self.py)
        f[y:y + 8, x:x + 8] = (187, 187, 53)
        for i in range(self.N_ENEMIES):
            ex, ey = int(self.ex[i]), int(self.ey[i])
            if 0 <= ey < self.H - 8:
                f[ey:ey + 8, ex:ex + 12] = (170, 170, 170) if i % 2 else (92, 186, 92)
        if self.bullet is not None:
            bx, by = int(self.bullet[0]), int(self.bullet[1])
            if 0 <= by < self.H - 4:
                f[by:by + 4, bx:bx + 2] = (214, 92, 92)
        return f.copy()

    def render(self, mode="rgb_array"):
        return self._frame.copy()


def register_atari(env_id: str) -> None:
    game = game_of(env_id)
    max_steps = 400000 if "NoFrameskip" in env_id else 100000
    register(env_id, lambda g=game: SyntheticAtariEnv(g), max_steps)


for _g in GAME_ACTIONS:
    register_atari(f"{_g}NoFrameskip-v4")


# ----------------------------------------------------------------------------------
# Reference-named wrapper adapters (origin_repo/wrapper.py API).  The preprocessing itself
# lives in :mod:`apex_amd.envs.preprocess` (one pipeline, AtariPreprocess); each class here
# only binds one of its stages into the gym-style wrapper composition the reference's
# callers use (make_atari / wrap_atari_dqn / wrap_deepmind).
# ----------------------------------------------------------------------------------
class NoopResetEnv(Wrapper):
    """Start stage: emulator reset + random no-op frames (``fixed_noops`` pins the count)."""

    def __init__(self, env, noop_max=30):
        super().__init__(env)
        if P.meaning(env, 0) != "NOOP":
            raise ValueError("NoopResetEnv needs NOOP at action 0")
        self.noop_max = noop_max
        self.fixed_noops = None

    def reset(self, **kwargs):
        return P.noop_start(self.env, self.noop_max, self.fixed_noops, kwargs)


class FireResetEnv(Wrapper):
    """FIRE start stage."""

    def __init__(self, env):
        super().__init__(env)
        if P.meaning(env, 1) != "FIRE" or len(env.unwrapped.get_action_meanings()) < 3:
            raise ValueError("FireResetEnv needs FIRE at action 1 and at least 3 actions")

    def reset(self, **kwargs):
        return P.fire_start(lambda: self.env.reset(**kwargs), self.env.step)


class EpisodicLifeEnv(Wrapper):
    """Life-ledger stage: a lost life ends the agent's episode; ``ledger.game_over`` says
    whether the next start must reset the emulator."""

    def __init__(self, env):
        super().__init__(env)
        self.ledger = P.LifeLedger()

    @property
    def lives(self):
        return self.ledger.lives

    def step(self, action):
        obs, reward, done, info = self.env.step(action)
        return obs, reward, self.ledger.observe(done, P.lives_of(self.env)), info

    def reset(self, **kwargs):
        return P.life_start(self.ledger, lambda: self.env.reset(**kwargs), self.env.step,
                            lambda: P.lives_of(self.env))


class MaxAndSkipEnv(Wrapper):
    """Repeat stage: ``skip`` frames per action, max-pooled over the persistent two-slot
    buffer of the reference (see ``preprocess.RepeatPool``)."""

    def __init__(self, env, skip=4):
        super().__init__(env)
        self.pool = P.RepeatPool(skip)

    def step(self, action):
        return self.pool.run(self.env.step, action)


class ClipRewardEnv(RewardWrapper):
    def reward(self, reward):
        return P.sign_reward(reward)


def _area_matrix(n_out: int, n_in: int) -> np.ndarray:
    return P.area_weights(n_out, n_in)


class WarpFrame(ObservationWrapper):
    """Resample stage: grey + area averaging to ``height x width`` (no OpenCV)."""

    def __init__(self, env, width=84, height=84, grayscale=True):
        super().__init__(env)
        self.resize = P.AreaResize(env.observation_space.shape[:2], (height, width), grayscale)
        self.observation_space = Box(0, 255, shape=(height, width, self.resize.channels), dtype=np.uint8)

    def observation(self, frame):
        return self.resize(frame)


class LazyFrames:
    """Frames shared between consecutive observations (wrapper.py:218-252)."""

    _axis = -1

    def __init__(self, frames):
        self._frames = frames
        self._out = None

    def _force(self):
        # ``_frames`` is kept after forcing (unlike wrapper.py:230) so the role actors can
        # ship each frame once (frame-id dedup, apex_amd.roles.common.FrameDedup)
        if self._out is None:
            self._out = np.concatenate(self._frames, axis=self._axis)
        return self._out

    def frames(self):
        return self._frames

    def __array__(self, dtype=None, copy=None):
        out = self._force()
        if dtype is not None:
            out = out.astype(dtype)
        return out

    def __len__(self):
        return len(self._force())

    def __getitem__(self, i):
        return self._force()[i]


class TorchLazyFrames(LazyFrames):
    _axis = 0


class FrameStack(Wrapper):
    """Stack stage: the last ``k`` frames as one LazyFrames (shared, not copied)."""

    lazy = LazyFrames

    def __init__(self, env, k):
        super().__init__(env)
        self.k = k
        self.frames = deque([], maxlen=k)
        shp = list(env.observation_space.shape)
        shp[self.lazy._axis] *= k
        self.observation_space = Box(0, 255, shape=tuple(shp), dtype=env.observation_space.dtype)

    def reset(self):
        first = self.env.reset()
        self.frames.extend([first] * self.k)
        return self.lazy(list(self.frames))

    def step(self, action):
        ob, reward, done, info = self.env.step(action)
        self.frames.append(ob)
        return self.lazy(list(self.frames)), reward, done, info


class TorchFrameStack(FrameStack):
    lazy = TorchLazyFrames


class ScaledFloatFrame(ObservationWrapper):
    def __init__(self, env):
        super().__init__(env)
        self.observation_space = Box(0, 1, shape=env.observation_space.shape, dtype=np.float32)

    def observation(self, observation):
        return np.asarray(observation, dtype=np.float32) / 255.0


class ImageToPyTorch(ObservationWrapper):
    """Layout stage: HWC -> CWH (H and W transposed)."""

    def __init__(self, env):
        super().__init__(env)
        h, w, c = self.observation_space.shape
        self.observation_space = Box(0, 255, shape=(c, h, w), dtype=np.uint8)

    def observation(self, observation):
        return P.channels_first(observation)


def make_atari(env_id, max_episode_steps=None):
    """Raw emulator + start and repeat stages (NoFrameskip ids only)."""
    from .core import make

    env = make(env_id)
    if "NoFrameskip" not in env.spec.id:
        raise ValueError(f"make_atari expects a NoFrameskip id, got {env_id}")
    env = MaxAndSkipEnv(NoopResetEnv(env, noop_max=30), skip=4)
    return TimeLimit(env, max_episode_steps=max_episode_steps) if max_episode_steps is not None else env


def _wrap(env, spec: P.PreprocessSpec, torch_layout: bool):
    """The pipeline stages of ``spec`` as a wrapper stack over a ``make_atari`` env."""
    if spec.episode_life:
        env = EpisodicLifeEnv(env)
    if P.has_fire(env) if spec.fire_reset is None else spec.fire_reset:
        env = FireResetEnv(env)
    env = WarpFrame(env)
    if spec.scale:
        env = ScaledFloatFrame(env)
    if spec.clip_rewards:
        env = ClipRewardEnv(env)
    if torch_layout:
        env = ImageToPyTorch(env)
    if spec.stack > 1:
        env = (TorchFrameStack if torch_layout else FrameStack)(env, spec.stack)
    return env


def wrap_deepmind(env, episode_life=True, clip_rewards=True, frame_stack=False, scale=False):
    spec = P.PreprocessSpec(episode_life=episode_life, clip_rewards=clip_rewards, stack=4 if frame_stack else 1,
                            scale=scale, channels_first=False)
    return _wrap(env, spec, torch_layout=False)


def wrap_atari_dqn(env, args):
    """The Ape-X actor's stack (origin_repo/actor.py:56-57): the reference flags of ``args``."""
    return _wrap(env, P.PreprocessSpec.from_args(args), torch_layout=True)


def make_preprocessed(env_id: str, n: int, spec: P.PreprocessSpec | None = None, seed: int | None = None):
    """N raw emulators of ``env_id`` under one :class:`~apex_amd.envs.preprocess.AtariPreprocess`."""
    from .core import make

    pipe = P.AtariPreprocess([make(env_id) for _ in range(n)], spec or P.PreprocessSpec())
    if seed is not None:
        pipe.seed(seed)
    return pipe
