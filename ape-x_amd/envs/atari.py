"""Atari-shaped environments and the DeepMind wrapper stack.

ALE / gym[atari] / OpenCV are not installed, so ``make_atari`` builds a seeded
*synthetic Atari emulator* with the same observable contract as an ALE
``*NoFrameskip-v4`` env: 210x160x3 uint8 RGB frames, the ALE action-meaning lists,
``ale.lives()``, ``np_random`` and raw (unclipped) game scores.  The wrapper classes
reproduce origin_repo/wrapper.py:11-329 behaviour (NoopReset, FireReset, EpisodicLife,
MaxAndSkip, ClipReward, WarpFrame, FrameStack/TorchFrameStack + LazyFrames,
ScaledFloatFrame, ImageToPyTorch, TimeLimit, make_atari, wrap_deepmind,
wrap_atari_dqn), with WarpFrame's grayscale + INTER_AREA resize implemented as a
separable area-averaging matrix product (no OpenCV).

The GPU-resident vector env used by the high-throughput engine
(`vec_env_step_k`, ops/csrc/actor_kernels.hip, driven by :mod:`apex_amd.engine.actor_shard`) renders the same game family straight to 84x84.
"""
from __future__ import annotations

from collections import deque

import numpy as np

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
# DeepMind wrappers (origin_repo/wrapper.py)
# ----------------------------------------------------------------------------------
class NoopResetEnv(Wrapper):
    def __init__(self, env, noop_max=30):
        super().__init__(env)
        self.noop_max = noop_max
        self.override_num_noops = None
        self.noop_action = 0
        assert env.unwrapped.get_action_meanings()[0] == "NOOP"

    def reset(self, **kwargs):
        self.env.reset(**kwargs)
        noops = self.override_num_noops if self.override_num_noops is not None else \
            self.unwrapped.np_random.randint(1, self.noop_max + 1)
        assert noops > 0
        obs = None
        for _ in range(noops):
            obs, _, done, _ = self.env.step(self.noop_action)
            if done:
                obs = self.env.reset(**kwargs)
        return obs


class FireResetEnv(Wrapper):
    def __init__(self, env):
        super().__init__(env)
        assert env.unwrapped.get_action_meanings()[1] == "FIRE"
        assert len(env.unwrapped.get_action_meanings()) >= 3

    def reset(self, **kwargs):
        self.env.reset(**kwargs)
        obs, _, done, _ = self.env.step(1)
        if done:
            self.env.reset(**kwargs)
        obs, _, done, _ = self.env.step(2)
        if done:
            self.env.reset(**kwargs)
        return obs


class EpisodicLifeEnv(Wrapper):
    def __init__(self, env):
        super().__init__(env)
        self.lives = 0
        self.was_real_done = True

    def step(self, action):
        obs, reward, done, info = self.env.step(action)
        self.was_real_done = done
        lives = self.env.unwrapped.ale.lives()
        if 0 < lives < self.lives:
            done = True
        self.lives = lives
        return obs, reward, done, info

    def reset(self, **kwargs):
        if self.was_real_done:
            obs = self.env.reset(**kwargs)
        else:
            obs, _, _, _ = self.env.step(0)
        self.lives = self.env.unwrapped.ale.lives()
        return obs


class MaxAndSkipEnv(Wrapper):
    def __init__(self, env, skip=4):
        super().__init__(env)
        self._obs_buffer = np.zeros((2,) + env.observation_space.shape, dtype=np.uint8)
        self._skip = skip

    def step(self, action):
        total_reward, done, info = 0.0, None, {}
        for i in range(self._skip):
            obs, reward, done, info = self.env.step(action)
            if i == self._skip - 2:
                self._obs_buffer[0] = obs
            if i == self._skip - 1:
                self._obs_buffer[1] = obs
            total_reward += reward
            if done:
                break
        return self._obs_buffer.max(axis=0), total_reward, done, info


class ClipRewardEnv(RewardWrapper):
    def reward(self, reward):
        return np.sign(reward)


def _area_matrix(n_out: int, n_in: int) -> np.ndarray:
    """Row-stochastic area-overlap weights (INTER_AREA downscale)."""
    scale = n_in / n_out
    m = np.zeros((n_out, n_in), dtype=np.float64)
    for o in range(n_out):
        lo, hi = o * scale, (o + 1) * scale
        for i in range(int(np.floor(lo)), min(int(np.ceil(hi)), n_in)):
            m[o, i] = max(0.0, min(hi, i + 1) - max(lo, i))
        m[o] /= m[o].sum()
    return m


class WarpFrame(ObservationWrapper):
    def __init__(self, env, width=84, height=84, grayscale=True):
        super().__init__(env)
        self.width, self.height, self.grayscale = width, height, grayscale
        c = 1 if grayscale else 3
        self.observation_space = Box(0, 255, shape=(height, width, c), dtype=np.uint8)
        h_in, w_in = env.observation_space.shape[:2]
        self._wy = _area_matrix(height, h_in)
        self._wx = _area_matrix(width, w_in).T

    def observation(self, frame):
        f = frame.astype(np.float64)
        if self.grayscale:
            f = f @ np.array([0.299, 0.587, 0.114])
            out = self._wy @ f @ self._wx
            return np.clip(np.rint(out), 0, 255).astype(np.uint8)[..., None]
        out = np.stack([self._wy @ f[..., k] @ self._wx for k in range(3)], -1)
        return np.clip(np.rint(out), 0, 255).astype(np.uint8)


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
    def __init__(self, env, k):
        super().__init__(env)
        self.k = k
        self.frames = deque([], maxlen=k)
        shp = env.observation_space.shape
        self.observation_space = Box(0, 255, shape=(shp[:-1] + (shp[-1] * k,)), dtype=env.observation_space.dtype)

    def reset(self):
        ob = self.env.reset()
        for _ in range(self.k):
            self.frames.append(ob)
        return self._get_ob()

    def step(self, action):
        ob, reward, done, info = self.env.step(action)
        self.frames.append(ob)
        return self._get_ob(), reward, done, info

    def _get_ob(self):
        assert len(self.frames) == self.k
        return LazyFrames(list(self.frames))


class TorchFrameStack(FrameStack):
    def __init__(self, env, k):
        super().__init__(env, k)
        shp = env.observation_space.shape
        self.observation_space = Box(0, 255, shape=((shp[0] * k,) + shp[1:]), dtype=env.observation_space.dtype)

    def _get_ob(self):
        assert len(self.frames) == self.k
        return TorchLazyFrames(list(self.frames))


class ScaledFloatFrame(ObservationWrapper):
    def __init__(self, env):
        super().__init__(env)
        self.observation_space = Box(0, 1, shape=env.observation_space.shape, dtype=np.float32)

    def observation(self, observation):
        return np.array(observation).astype(np.float32) / 255.0


class ImageToPyTorch(ObservationWrapper):
    """HWC -> CWH via swapaxes(2, 0) (H and W transposed)."""

    def __init__(self, env):
        super().__init__(env)
        old = self.observation_space.shape
        self.observation_space = Box(0, 255, shape=(old[-1], old[0], old[1]), dtype=np.uint8)

    def observation(self, observation):
        return np.swapaxes(observation, 2, 0)


def make_atari(env_id, max_episode_steps=None):
    from .core import make

    env = make(env_id)
    assert "NoFrameskip" in env.spec.id
    env = NoopResetEnv(env, noop_max=30)
    env = MaxAndSkipEnv(env, skip=4)
    if max_episode_steps is not None:
        env = TimeLimit(env, max_episode_steps=max_episode_steps)
    return env


def wrap_deepmind(env, episode_life=True, clip_rewards=True, frame_stack=False, scale=False):
    if episode_life:
        env = EpisodicLifeEnv(env)
    if "FIRE" in env.unwrapped.get_action_meanings():
        env = FireResetEnv(env)
    env = WarpFrame(env)
    if scale:
        env = ScaledFloatFrame(env)
    if clip_rewards:
        env = ClipRewardEnv(env)
    if frame_stack:
        env = FrameStack(env, 4)
    return env


def wrap_atari_dqn(env, args):
    if args.episode_life:
        env = EpisodicLifeEnv(env)
    if "FIRE" in env.unwrapped.get_action_meanings():
        env = FireResetEnv(env)
    env = WarpFrame(env)
    if args.scale:
        env = ScaledFloatFrame(env)
    if args.clip_rewards:
        env = ClipRewardEnv(env)
    env = ImageToPyTorch(env)
    if args.frame_stack:
        env = TorchFrameStack(env, 4)
    return env
