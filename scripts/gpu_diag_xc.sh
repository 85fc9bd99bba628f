set -o pipefail
export RAFIKI_TUNE_CACHE=off
timeout -k 10 200 python -u scripts/diag_xconv_engine.py 2>&1 | grep -v amdgpu.ids
RAFIKI_XCONV=0 timeout -k 10 200 python -u scripts/diag_xconv_engine.py 2>&1 | grep -v amdgpu.ids
