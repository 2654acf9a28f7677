"""GPU-resident Ape-X engine (one rank = actor shard + HBM replay + learner)."""
