set -o pipefail
for t in 32,64 16,64 16,128 8,128 8,256 4,256 4,512; do
  timeout -k 10 120 python -u scripts/diag_xconv_layer.py $t 2>&1 | grep "xconv at" || exit 1
done
