# Same-box A/B of two kernel libraries on the shipped tune database (the VGG-small training step):
#   bash scripts/dev/ab_lib.sh <tag> <lib B> [rounds]     A = the in-tree rafiki_amd/_native/librafiki_kernels.so
# -> gpurun_out/ab_<tag>/results.txt : ms/step per run, A B A B ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; LIBB=$2; N=${3:-2}
O=gpurun_out/ab_$TAG
mkdir -p $O
run() {
  local name="$1" lib="$2" i="$3"
  RAFIKI_KERNEL_LIB=$lib timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --trials 0 --probe-trials 0 \
    --no-serving --configs none > $O/$name$i.log 2>&1 || { tail -5 $O/$name$i.log; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$name$i.log').read().strip().splitlines()[-1]); print('%s%d %.4f ms  %.0f img/s' % ('$name', $i, d['ms_per_step'], d['value']))" >> $O/results.txt
}
for i in $(seq 1 $N); do
  run a "$PWD/rafiki_amd/_native/librafiki_kernels.so" $i || exit 1
  run b "$PWD/$LIBB" $i || exit 1
done
cat $O/results.txt
