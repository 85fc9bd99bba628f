# Round-3 profiling pass: VGG-small step (kernel trace + PMC), PG-GAN lod 0 / lod 3 profiles,
# predictor QPS (native / asyncio HTTP front ends, in-process batcher)
set -o pipefail
mkdir -p gpurun_out/r3d
bash scripts/pmc_step.sh > gpurun_out/r3d/pmc_step.log 2>&1 || exit $?
cp -r gpurun_out/pmc_step gpurun_out/r3d/ && head -45 gpurun_out/r3d/pmc_step/summary.txt | cut -c1-150
bash scripts/gpu_pggan_prof.sh 0 4 > gpurun_out/r3d/pg0.log 2>&1 || exit $?
tail -45 gpurun_out/r3d/pg0.log | cut -c1-150
bash scripts/gpu_pggan_prof.sh 3 8 > gpurun_out/r3d/pg3.log 2>&1 || exit $?
tail -30 gpurun_out/r3d/pg3.log | cut -c1-150
timeout -k 10 300 python -u scripts/bench_predictor.py --out gpurun_out/r3d/predictor_qps.json > gpurun_out/r3d/qps.log 2>&1 || exit $?
tail -1 gpurun_out/r3d/qps.log | cut -c1-1500
