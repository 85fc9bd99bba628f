# x6p counter passes (scripts/pmc_x6p.sh) over the 64x64 / 128x128 / warp-specialised tiles, with and
# without the DMA (RAFIKI_X6P_DBG=1)
set -o pipefail
for a in "c5f 3,2,1 0" "c5f 3,2,1 1" "c5f 0,2,1 1" "c5f 12,3,1 0" "c7f 8,2,1 0"; do
  echo "== $a"
  timeout -k 10 200 bash scripts/pmc_x6p.sh $a || { echo "fail $a"; exit 1; }
done
