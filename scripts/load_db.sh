#!/usr/bin/env bash
# Restore the metadata store from a dump made by save_db.sh (reference scripts/load_db.sh).
set -euo pipefail
cd "$(dirname "$0")/.."
source ./env.sh
dump="${1:-$WORKDIR_PATH/db_dump.sqlite3}"
if [[ ! -f "$dump" ]]; then echo "no dump at $dump, skipping"; exit 0; fi
python - "$dump" "$WORKDIR_PATH/rafiki.sqlite3" <<'PY'
import sqlite3, sys
src, dst = sqlite3.connect(sys.argv[1]), sqlite3.connect(sys.argv[2])
src.backup(dst); dst.close(); src.close(); print('loaded', sys.argv[1])
PY
