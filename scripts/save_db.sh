#!/usr/bin/env bash
# Checkpoint the metadata store (reference scripts/save_db.sh used pg_dump): consistent online
# SQLite backup to $WORKDIR_PATH/db_dump.sqlite3 (or $1).
set -euo pipefail
cd "$(dirname "$0")/.."
source ./env.sh
python - "$WORKDIR_PATH/rafiki.sqlite3" "${1:-$WORKDIR_PATH/db_dump.sqlite3}" <<'PY'
import sqlite3, sys
src, dst = sqlite3.connect(sys.argv[1]), sqlite3.connect(sys.argv[2])
src.backup(dst); dst.close(); src.close(); print('saved', sys.argv[2])
PY
