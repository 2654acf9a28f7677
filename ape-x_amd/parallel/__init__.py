"""Multi-GPU layer over torch.distributed (``nccl`` = RCCL over xGMI on MI355X,
``gloo`` for CPU tests): data-parallel gradient all-reduce, versioned parameter
broadcast, actor->replay experience push, sharded-replay global sampling, rank
heartbeats / fault injection."""
from .broadcast import ParamPublisher, ParamSubscriber, broadcast_flat
from .dp import FlatGradAllReduce, allreduce_mean_

__all__ = ["ParamPublisher", "ParamSubscriber", "broadcast_flat", "FlatGradAllReduce", "allreduce_mean_"]
