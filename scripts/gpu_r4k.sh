# r4k: PG-GAN tests + lod-3 profile after the penalty / in-place changes; VGG step counters (pmc_step)
set -o pipefail
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_pg_gan_gpu.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 bash scripts/gpu_pggan_prof.sh 3 6 > $O/pg3.log 2>&1 || { tail -5 $O/pg3.log; exit 1; }
head -3 gpurun_out/pgprof_lod3/kernels.txt; grep "at::native" gpurun_out/pgprof_lod3/kernels.txt | head -5; tail -1 gpurun_out/pgprof_lod3/pmc.txt
timeout -k 10 900 bash scripts/pmc_step.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
tail -3 $O/pmc.log
