#!/usr/bin/env bash
# Remove runtime state: logs, params, run files, the SQLite store and build outputs (reference scripts/clean.sh).
set -euo pipefail
cd "$(dirname "$0")/.."
source ./env.sh
rm -rf "$WORKDIR_PATH/logs" "$WORKDIR_PATH/params" "$WORKDIR_PATH/run" "$WORKDIR_PATH/rafiki.sqlite3"* build/
echo "cleaned $WORKDIR_PATH"
