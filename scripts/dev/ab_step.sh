# A/B of step-level switches on ONE box with ONE tune database (captured by the first run):
#   bash scripts/dev/ab_step.sh <tag> "ENV=VAL ..." ["ENV=VAL ..."] ...   (the first spec is the baseline; "-" = none)
# -> gpurun_out/ab_<tag>/results.txt : ms/step per spec, baseline repeated last to show the run-to-run noise
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
O=gpurun_out/ab_$TAG
mkdir -p $O
export RAFIKI_TUNE_CACHE=$PWD/$O/tune_db.json
run() {
  local spec="$1" i="$2"
  [ "$spec" = "-" ] && spec=""
  env $spec timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 --trials 0 --probe-trials 0 --no-serving --configs none \
    > $O/run$i.log 2>&1 || { tail -5 $O/run$i.log; return 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/run$i.log').read().strip().splitlines()[-1]); print('%-40s %.4f ms  %.0f img/s' % ('$spec' or 'baseline', d['ms_per_step'], d['value']))" >> $O/results.txt
}
i=0
for spec in "$@" "$1"; do
  run "$spec" $i || exit 1
  i=$((i+1))
done
cat $O/results.txt
