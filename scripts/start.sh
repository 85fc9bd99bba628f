#!/usr/bin/env bash
# Bring up the static stack (reference scripts/start.sh): build the native libraries, then start
# the admin (which seeds the superadmin and launches workers/predictors on demand) and the advisor.
set -euo pipefail
cd "$(dirname "$0")/.."
source ./env.sh
mkdir -p "$WORKDIR_PATH/logs" "$WORKDIR_PATH/run"
python -m rafiki_amd._build
start() {  # name module
  local pidf="$WORKDIR_PATH/run/$1.pid"
  if [[ -f "$pidf" ]] && kill -0 "$(cat "$pidf")" 2>/dev/null; then echo "$1 already running"; return; fi
  nohup python -m "$2" > "$WORKDIR_PATH/logs/$1.out" 2>&1 &
  echo $! > "$pidf"
  echo "started $1 (pid $!)"
}
start admin rafiki_amd.admin
start advisor rafiki_amd.advisor
for i in $(seq 1 60); do
  if python - <<PY 2>/dev/null; then break; fi
import urllib.request; urllib.request.urlopen('http://$ADMIN_HOST:$ADMIN_PORT/', timeout=1)
PY
  sleep 1
done
echo "Admin on http://$ADMIN_HOST:$ADMIN_PORT (web UI at /ui); use rafiki_amd.client.Client from Python."
