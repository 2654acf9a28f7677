#!/bin/bash
# Evaluator host (origin_repo/deploy/evaluator.sh): greedy, unclipped rewards.
source "$(dirname "$0")/_common.sh"
export N_ACTORS=$((N_NODE * ACTOR_PER_NODE))
start_role evaluator python -m apex_amd.roles.evaluator "$@"
