#!/bin/bash
# A/B of sgemm diagnostics variants on one config: scripts/sgemm_dbg.sh <layer> <pass> <tile> <nst> <splits>
set -e -o pipefail
for d in 0 1 2 3; do
  RAFIKI_SGEMM_DBG=$d timeout -k 10 60 python3 scripts/prof_sgemm_one.py "$1" "$2" "$3" "$4" "${5:-1}" 100 2>&1 | grep -v amdgpu | sed "s/^/dbg=$d /"
done
