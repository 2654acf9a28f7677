#!/bin/bash
# Actor host NODE_ID of N_NODE (origin_repo/deploy/actor.sh): ACTOR_PER_NODE actors,
# global ids NODE_ID * ACTOR_PER_NODE + i, so the epsilon ladder spans the cluster.
source "$(dirname "$0")/_common.sh"
: "${NODE_ID:?set NODE_ID (0 .. N_NODE-1)}"
export N_ACTORS=$((N_NODE * ACTOR_PER_NODE))
for ((i = 0; i < ACTOR_PER_NODE; i++)); do
  ACTOR_ID=$((NODE_ID * ACTOR_PER_NODE + i)) start_role "actor-$((NODE_ID * ACTOR_PER_NODE + i))" \
    python -m apex_amd.roles.actor "$@"
done
