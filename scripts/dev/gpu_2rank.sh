set -o pipefail
mkdir -p gpurun_out
RAFIKI_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/bench_2rank.log 2>&1
rc=$?
grep '^{' gpurun_out/bench_2rank.log | cut -c1-1200
exit $rc
