set -o pipefail
mkdir -p gpurun_out
bash scripts/pmc_wino.sh w4f32 256 32 64 64 fwd4 0 > gpurun_out/pmc_w4f32.log 2>&1 && \
bash scripts/pmc_wino.sh w4g32 256 32 64 64 wgrad4 128 > gpurun_out/pmc_w4g32.log 2>&1 && \
bash scripts/pmc_wino.sh w4g4 256 4 512 512 wgrad4 2 > gpurun_out/pmc_w4g4.log 2>&1 && \
bash scripts/pmc_wino.sh w2f32 256 32 64 64 fwd > gpurun_out/pmc_w2f32.log 2>&1
rc=$?
for f in w4f32 w4g32 w4g4 w2f32; do echo "== $f"; cat gpurun_out/pmc_$f/summary.txt; done
exit $rc
