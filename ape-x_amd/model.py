"""Reference-compatible ``model`` module (reference model.py)."""
from .models.aql import AQL, Proposal_Network, Q_Network  # noqa: F401
from .models.dqn import DuelingDQN, Flatten, init, init_  # noqa: F401
from .models.noisy import NoisyLinear  # noqa: F401
