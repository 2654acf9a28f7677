#!/bin/bash
# Stop the roles started on this host by deploy/*.sh (exact PIDs from $LOG_DIR/*.pid).
source "$(dirname "$0")/_common.sh"
for f in "$LOG_DIR"/*.pid; do
  [ -e "$f" ] || continue
  pid=$(cat "$f")
  if kill -0 "$pid" 2>/dev/null; then
    echo "[deploy] stopping $(basename "$f" .pid) ($pid)"
    kill "$pid"
  fi
  rm -f "$f"
done
