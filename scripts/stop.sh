#!/usr/bin/env bash
# Stop all jobs, then the admin and advisor (reference scripts/stop.sh).  Processes are stopped by
# the exact PIDs recorded at start-up.
set -uo pipefail
cd "$(dirname "$0")/.."
source ./env.sh
python scripts/stop_all_jobs.py 2>/dev/null || true
for name in advisor admin; do
  pidf="$WORKDIR_PATH/run/$name.pid"
  if [[ -f "$pidf" ]]; then
    pid=$(cat "$pidf")
    kill "$pid" 2>/dev/null && echo "stopped $name ($pid)"
    rm -f "$pidf"
  fi
done
