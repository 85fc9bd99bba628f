# Round-3 pass 2: new-kernel tests, per-layer pt benches, VGG-small step profile (kernel trace + PMC),
# PG-GAN lod 0 / 3 profiles, predictor QPS
set -o pipefail
mkdir -p gpurun_out/r3d
timeout -k 10 300 python -u -m pytest tests/test_winograd4_gpu.py -q -k "pretransformed" --timeout 120 --timeout-method thread > gpurun_out/r3d/pt_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3d/pt_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/bench_conv_pt.py gpurun_out/r3d/conv_pt.jsonl > gpurun_out/r3d/conv_pt.log 2>&1 || exit $?
cut -c1-200 gpurun_out/r3d/conv_pt.log
timeout -k 10 200 python -u scripts/diag_pggan_det.py > gpurun_out/r3d/det.log 2>&1; cat gpurun_out/r3d/det.log | tail -40
timeout -k 10 300 python -u bench.py --trials 0 --probe-trials 0 --no-serving > gpurun_out/r3d/bench_quick.log 2>&1 || exit $?
tail -1 gpurun_out/r3d/bench_quick.log | cut -c1-300
bash scripts/pmc_step.sh > gpurun_out/r3d/pmc_step.log 2>&1 || exit $?
cp -r gpurun_out/pmc_step gpurun_out/r3d/ && head -40 gpurun_out/r3d/pmc_step/summary.txt | cut -c1-150
bash scripts/gpu_pggan_prof.sh 0 4 > gpurun_out/r3d/pg0.log 2>&1 || exit $?
tail -45 gpurun_out/r3d/pg0.log | cut -c1-150
bash scripts/gpu_pggan_prof.sh 3 8 > gpurun_out/r3d/pg3.log 2>&1 || exit $?
tail -30 gpurun_out/r3d/pg3.log | cut -c1-150
