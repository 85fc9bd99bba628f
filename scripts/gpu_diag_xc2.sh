set -o pipefail
export RAFIKI_TUNE_CACHE=off
for cfg in "RAFIKI_XCONV=fwd" "RAFIKI_XCONV=dgrad"; do
  env $cfg timeout -k 10 200 python -u scripts/diag_f32_grads.py > gpurun_out/diag/out.log 2>&1 || { tail -5 gpurun_out/diag/out.log; exit 1; }
  grep -E "^X6|conv6.gamma|conv7|conv5.gamma|conv3" gpurun_out/diag/out.log ; grep "tune" gpurun_out/diag/out.log | grep -- "-3[0-4]"
done
