# PG-GAN resampling-conv weights as one batched GEMM: PG-GAN GPU tests, bench, lod-0 kernel trace
set -o pipefail
mkdir -p gpurun_out/r3p
timeout -k 10 500 python -u -m pytest tests/test_pg_gan_gpu.py tests/test_resample_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r3p/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3p/tests.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_pg_gan.py --lods 3,0 > gpurun_out/r3p/pg.log 2>&1 || exit $?
tail -1 gpurun_out/r3p/pg.log | cut -c150-600
bash scripts/gpu_pggan_prof.sh 0 > gpurun_out/r3p/pgprof.log 2>&1 || { tail -5 gpurun_out/r3p/pgprof.log; exit 1; }
grep -E "wall/step|at::native" gpurun_out/pgprof_lod0/kernels.txt | head -12 | cut -c1-150
