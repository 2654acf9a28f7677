"""Replay: reference-API host buffers (native trees) and the HBM/GPU replay."""
from .buffers import (CustomPrioritizedReplayBuffer, CustomPrioritizedReplayBuffer_AQL, PrioritizedReplayBuffer,
                      ReplayBuffer)
from .nstep import BatchStorage
from .segment_tree import MinSegmentTree, SegmentTree, SumSegmentTree

__all__ = ["ReplayBuffer", "PrioritizedReplayBuffer", "CustomPrioritizedReplayBuffer",
           "CustomPrioritizedReplayBuffer_AQL", "BatchStorage", "SegmentTree", "SumSegmentTree", "MinSegmentTree"]
