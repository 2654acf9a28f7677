#!/bin/bash
# Replay server host (origin_repo/deploy/replay.sh).  Start it first: it hosts the
# TCPStore rendezvous every other role connects to (REPLAY_IP:APEX_PORT).
source "$(dirname "$0")/_common.sh"
export N_ACTORS=$((N_NODE * ACTOR_PER_NODE))
start_role replay python -m apex_amd.roles.replay "$@"
