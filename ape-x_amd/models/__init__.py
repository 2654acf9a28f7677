"""Model families: Dueling (double) DQN with Nature-CNN / MLP trunk, NoisyNet layer,
and the AQL action-proposal model.  HIP fast paths: :mod:`apex_amd.models.fused`."""
from .aql import AQL, Proposal_Network, Q_Network
from .dqn import DuelingDQN, Flatten, env_spec, init, init_
from .noisy import NoisyLinear

__all__ = ["AQL", "Proposal_Network", "Q_Network", "DuelingDQN", "Flatten", "env_spec", "init", "init_",
           "NoisyLinear"]
