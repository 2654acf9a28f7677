# Shared helpers for deploy/*.sh (sourced).
DEPLOY_DIR="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
REPO_ROOT="$(dirname "$DEPLOY_DIR")"
# shellcheck source=cluster.env
source "$DEPLOY_DIR/cluster.env"
export PYTHONPATH="$REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
LOG_DIR=${LOG_DIR:-$REPO_ROOT/logs}
mkdir -p "$LOG_DIR"

# start_role NAME CMD...: run in the background, log to $LOG_DIR/NAME.log, record the PID
start_role() {
  local name=$1; shift
  echo "[deploy] $name: $*" | tee -a "$LOG_DIR/deploy.log"
  nohup "$@" > "$LOG_DIR/$name.log" 2>&1 &
  echo $! > "$LOG_DIR/$name.pid"
}
