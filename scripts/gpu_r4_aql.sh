#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/ab/aql_bwd_tree.sh
