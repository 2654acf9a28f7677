"""Reference-compatible ``wrapper`` module (origin_repo/wrapper.py)."""
from .envs.atari import (ClipRewardEnv, EpisodicLifeEnv, FireResetEnv, FrameStack, ImageToPyTorch,  # noqa: F401
                         LazyFrames, MaxAndSkipEnv, NoopResetEnv, ScaledFloatFrame, TorchFrameStack, TorchLazyFrames,
                         WarpFrame, make_atari, wrap_atari_dqn, wrap_deepmind)
from .envs.core import TimeLimit  # noqa: F401
