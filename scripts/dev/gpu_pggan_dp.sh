# PG-GAN data-parallel round on a 1-rank RCCL group (segmented graphs around eager bucketed all-reduces):
# throughput at LOD 3 / 0 next to the plain graphed round, and the per-round kernel list at LOD 3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pgdp
mkdir -p $O
timeout -k 10 600 python3 -u scripts/bench_pg_gan.py --lods 3,0 --steps 10 --force-allreduce > $O/dp.log 2>&1 || { tail -20 $O/dp.log; exit 1; }
tail -1 $O/dp.log | cut -c1-700
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- \
  python3 scripts/bench_pg_gan.py --lods 3 --steps 6 --warmup 3 --force-allreduce > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
python3 scripts/trace_steps.py $(find $O/t -name '*kernel_trace.csv' | head -1) --steps 6 --marker lerp_ \
  --csv $O/kernels.csv --seq $O/seq.txt > $O/kernels.txt
rm -rf $O/t
head -25 $O/kernels.txt
