# driver rehearsal at HEAD: build check import, smoke, the 2-rank torchrun path (gloo on one GPU), bench --gpus 1
set -o pipefail
mkdir -p gpurun_out/r3q
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3q/smoke.log 2>&1 || { tail -5 gpurun_out/r3q/smoke.log; exit 1; }
tail -1 gpurun_out/r3q/smoke.log
RAFIKI_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --trials 1 --probe-trials 2 > gpurun_out/r3q/bench_2rank.log 2>&1 || { tail -5 gpurun_out/r3q/bench_2rank.log; exit 1; }
grep '^{' gpurun_out/r3q/bench_2rank.log | cut -c1-700
timeout -k 10 400 python -u bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/r3q/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3q/bench.log | cut -c1-400
