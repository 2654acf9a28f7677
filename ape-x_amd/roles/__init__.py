"""Role processes of the distributed Ape-X topology.

``replay`` (rank 0, hosts the rendezvous store) / ``learner`` (rank 1) /
``evaluator`` (rank 2) / ``actor`` (ranks 3..) talk over ``torch.distributed``
point-to-point messages (:mod:`.wire`) and a versioned parameter channel
(:mod:`.common`), replacing the reference's ZeroMQ sockets and pickles.  ``enjoy``
plays a checkpoint.  Every role accepts the reference ``arguments.py`` flags and the
``ACTOR_ID`` / ``N_ACTORS`` / ``REPLAY_IP`` / ``LEARNER_IP`` env vars; ``launch``
starts a whole single-host job (the reference's ``run.sh``).
"""
