set -o pipefail
mkdir -p gpurun_out/diag
export RAFIKI_TUNE_CACHE=off
for cfg in "RAFIKI_X6=0" "RAFIKI_X6=1 RAFIKI_XCONV=0 RAFIKI_PT_MAX_HW=8" "RAFIKI_X6=1 RAFIKI_XCONV=0" "RAFIKI_X6=1 RAFIKI_PT_MAX_HW=8" "RAFIKI_X6=1"; do
  env $cfg timeout -k 10 200 python -u scripts/diag_f32_grads.py > gpurun_out/diag/out.log 2>&1 || { tail -5 gpurun_out/diag/out.log; exit 1; }
  cat gpurun_out/diag/out.log | grep -v "^  tune" ; grep "^  tune" gpurun_out/diag/out.log | head -30
done
