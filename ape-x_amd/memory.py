"""Reference-compatible ``memory`` module (reference memory.py)."""
from .replay.buffers import (CustomPrioritizedReplayBuffer, CustomPrioritizedReplayBuffer_AQL,  # noqa: F401
                             PrioritizedReplayBuffer, ReplayBuffer)
from .replay.nstep import BatchStorage  # noqa: F401
from .replay.segment_tree import MinSegmentTree, SegmentTree, SumSegmentTree  # noqa: F401
