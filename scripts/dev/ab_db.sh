#!/bin/bash
# A/B of two shipped tune databases on ONE box: bash scripts/dev/ab_db.sh A.json B.json  (runs A B A B)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_db; mkdir -p $O
DST=rafiki_amd/tune/$(python3 -c "from rafiki_amd.ops import autotune; print(autotune.db_name())")
export RAFIKI_TUNE_CACHE=off
i=0
for db in "$1" "$2" "$1" "$2"; do
  cp "$db" "$DST"
  timeout -k 10 400 python -u bench.py --steps 50 --warmup 10 --trials 0 --probe-trials 0 --no-serving \
    > $O/run$i.log 2>&1 || { tail -5 $O/run$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/run$i.log').read().strip().splitlines()[-1]); print('%-24s %.4f ms  %.0f img/s' % ('$db', d['ms_per_step'], d['value']))" | tee -a $O/results.txt
  i=$((i+1))
done
