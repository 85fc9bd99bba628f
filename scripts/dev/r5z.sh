#!/bin/bash
# vectorised column sums: tests, then the PG-GAN bench at lods 3 / 0
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5z; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_f32_gpu.py tests/test_pg_gan_gpu.py \
  > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/bench_pg_gan.py --lods 3,0 --steps 10 --warmup 3 > $O/pgbench.log 2>&1
rc=$?; tail -4 $O/pgbench.log | cut -c1-400; exit $rc
