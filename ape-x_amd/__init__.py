"""apex_amd -- MI355X-native Ape-X / DQN / AQL distributed prioritized-replay engine.

Layers (SURVEY.md §1 mapped to this package):

* ``envs``      gym-API envs, synthetic Atari + DeepMind wrappers (L0)
* ``models``    DuelingDQN / NoisyLinear / AQL with reference state_dict keys (L1)
* ``replay``    segment trees, PER buffers, n-step batcher (host, native C++) (L2/L3)
* ``algo``      double-DQN Huber loss, priorities, update, schedules (L3)
* ``ops``       native libraries: ``_apex_cpu`` (C++) and ``_apex_hip`` (gfx950 HIP)
* ``engine``    GPU-resident Ape-X: HBM replay, vector env, fused learner, HIP graphs
* ``parallel``  torch.distributed/RCCL: param broadcast, experience push, DP, sharded PER
* ``roles``     actor / replay / learner / eval / enjoy role entry points (L5)
* ``trainers``  single-node trainers: DQN, ApeX, AQL, AQL_dis (L5)
* ``config``    dataclass config tree + reference flag parser (L6)

``apex_amd.model`` / ``apex_amd.memory`` / ``apex_amd.utils`` mirror the reference's
top-level modules for drop-in use.
"""
__version__ = "0.1.0"
