#!/bin/bash
# Learner host (origin_repo/deploy/learner.sh): one MI355X runs the fused learner.
source "$(dirname "$0")/_common.sh"
export N_ACTORS=$((N_NODE * ACTOR_PER_NODE))
start_role learner python -m apex_amd.roles.learner --cuda "$@"
