# Round-3 pass 3: resampling-conv paths (tests, PG-GAN bench both modes), pt conv tests, VGG bench,
# predictor QPS, PG-GAN determinism diag
set -o pipefail
mkdir -p gpurun_out/r3e
timeout -k 10 300 python -u -m pytest tests/test_pg_gan_gpu.py tests/test_winograd4_gpu.py -q -k "resampling_conv_paths or pretransformed" --timeout 120 --timeout-method thread > gpurun_out/r3e/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3e/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_pg_gan.py --lods 3,0 > gpurun_out/r3e/pg_wino.log 2>&1 || exit $?
tail -1 gpurun_out/r3e/pg_wino.log
RAFIKI_PGGAN_RESAMPLE=direct timeout -k 10 300 python -u scripts/bench_pg_gan.py --lods 0 > gpurun_out/r3e/pg_direct.log 2>&1 || exit $?
tail -1 gpurun_out/r3e/pg_direct.log
timeout -k 10 300 python -u bench.py --trials 0 --probe-trials 0 --no-serving > gpurun_out/r3e/bench_quick.log 2>&1 || exit $?
tail -1 gpurun_out/r3e/bench_quick.log | cut -c1-200
timeout -k 10 400 python -u scripts/bench_predictor.py --out gpurun_out/r3e/predictor_qps.json > gpurun_out/r3e/qps.log 2>&1 || exit $?
tail -1 gpurun_out/r3e/qps.log | cut -c1-2000
timeout -k 10 200 python -u scripts/diag_pggan_det.py > gpurun_out/r3e/det.log 2>&1; tail -60 gpurun_out/r3e/det.log
