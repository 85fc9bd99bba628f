# Same-box A/B of environment switches on the PG-GAN rounds (scripts/bench_pg_gan.py), one tune database
# shared by every run (seeded by the shipped one; shapes it lacks are tuned by the first run that meets them):
#   bash scripts/dev/ab_pggan.sh <tag> "ENV=VAL ..." "ENV=VAL ..." [rounds]    ("-" = no switch)
# -> gpurun_out/abpg_<tag>/results.txt : ms per round at lod 3 and lod 0 per run, alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; A=$2; B=$3; N=${4:-2}
O=gpurun_out/abpg_$TAG
mkdir -p $O
export RAFIKI_TUNE_CACHE=$PWD/$O/tune_db.json
run() {
  local name="$1" spec="$2" i="$3"
  [ "$spec" = "-" ] && spec=""
  env $spec timeout -k 10 400 python -u scripts/bench_pg_gan.py --lods 3,0 --steps 20 --warmup 3 \
    > $O/$name$i.log 2>&1 || { tail -5 $O/$name$i.log; return 1; }
  python3 -c "
import json
d = json.loads([l for l in open('$O/$name$i.log') if l.startswith('{')][-1])
print('%s%d %-24s' % ('$name', $i, '$spec' or 'baseline'), ' '.join('lod%s %.3f ms' % (k, v['ms_per_round']) for k, v in d['lods'].items()))
" >> $O/results.txt
}
for i in $(seq 1 $N); do
  run a "$A" $i || exit 1
  run b "$B" $i || exit 1
done
cat $O/results.txt
