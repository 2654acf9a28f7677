"""Reference-equivalent trainers.

* :mod:`.dqn`            -- DQN.py (single-process prioritized double-DQN, CartPole)
* :mod:`.apex_single`    -- ApeX.py (single-node Ape-X with CPU actor workers)
* :mod:`.aql`            -- AQL.py / AQL_dis.py (amortized Q-learning)
* :mod:`.batchrecorder`  -- batchrecorder.py / batchrecoder_AQL.py (actor workers)

The GPU-resident Ape-X engine (vectorised actors + HBM replay + HIP learner) is
:mod:`apex_amd.engine`; the distributed role CLIs are :mod:`apex_amd.roles`.
"""
