#!/usr/bin/env bash
# Interleaved same-box A/B of bench.py configurations.  Each arg is "label:ENV=V,ENV2=V2" (env may
# be empty: "base:").  Rounds run every config once in order; prints one line per run.
#   bash scripts/dev/ab_bench.sh 2 "head:RAFIKI_KERNEL_LIB=ab/libhead.so" "new:"
set -uo pipefail
rounds=${1:?rounds}; shift
mkdir -p gpurun_out
for r in $(seq 1 "$rounds"); do
  for spec in "$@"; do
    label=${spec%%:*}; envs=${spec#*:}
    IFS=',' read -ra kv <<< "$envs"
    out=gpurun_out/ab_${label}_$r.log
    env "${kv[@]}" timeout -k 10 240 python bench.py --steps 100 --warmup 10 > "$out" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$label round $r FAILED rc=$rc"; tail -5 "$out"; exit $rc; fi
    python - "$out" "$label" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split('\n')[-1])
print(f"{sys.argv[2]:>12s} {d['value']:10.1f} img/s {d['ms_per_step']:.4f} ms")
PY
  done
done
