"""Environments: gym-API classic control, synthetic Atari + DeepMind wrappers.

``apex_amd.envs.make(id)`` is the ``gym.make`` of this framework.  The GPU-resident
vectorised Atari env for the engine is the `vec_env_*` HIP kernels (ops/csrc/actor_kernels.hip) driven by :mod:`apex_amd.engine.actor_shard`.
"""
from . import spaces
from .core import Env, EnvSpec, ObservationWrapper, RewardWrapper, TimeLimit, Wrapper, make, register, registered
from . import classic  # noqa: F401  (registers envs)
from . import atari  # noqa: F401
from .atari import (ClipRewardEnv, EpisodicLifeEnv, FireResetEnv, FrameStack, ImageToPyTorch, LazyFrames,
                    MaxAndSkipEnv, NoopResetEnv, ScaledFloatFrame, SyntheticAtariEnv, TorchFrameStack,
                    TorchLazyFrames, WarpFrame, make_atari, wrap_atari_dqn, wrap_deepmind)

__all__ = [
    "spaces", "Env", "EnvSpec", "Wrapper", "ObservationWrapper", "RewardWrapper", "TimeLimit", "make", "register",
    "registered", "ClipRewardEnv", "EpisodicLifeEnv", "FireResetEnv", "FrameStack", "ImageToPyTorch", "LazyFrames",
    "MaxAndSkipEnv", "NoopResetEnv", "ScaledFloatFrame", "SyntheticAtariEnv", "TorchFrameStack", "TorchLazyFrames",
    "WarpFrame", "make_atari", "wrap_atari_dqn", "wrap_deepmind",
]
