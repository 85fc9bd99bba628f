# Re-tune the PG-GAN large-map F(4x4) weight-gradient picks (16x16 / 32x32, 512 channels) against the shipped
# database, then A/B the PG-GAN rounds on the re-tuned database vs the shipped one (same box, A B A B).
#   bash scripts/dev/retune_pggan_wgrad.sh   -> gpurun_out/rt/{db.json, ab.txt}
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/rt
mkdir -p $O /tmp/shipped_seed_rt
python3 - <<'PY'
import glob, json
src = glob.glob('rafiki_amd/tune/*.json')[0]
d = json.load(open(src))
keep = {k: v for k, v in d.items()
        if not (json.loads(k)[0] == 'sw' and json.loads(k)[6] == 512 and json.loads(k)[7] == 9 and json.loads(k)[4] in (16, 32))}
print('dropped', len(d) - len(keep))
json.dump(keep, open('gpurun_out/rt/db.json', 'w'))
PY
mv rafiki_amd/tune/*.json /tmp/shipped_seed_rt/
export RAFIKI_TUNE_CACHE=$PWD/$O/db.json
for mb in 64 32 16 8; do
  timeout -k 10 300 python scripts/bench_pg_gan.py --lods 0 --minibatch $mb --steps 2 --warmup 2 >> $O/tune.jsonl 2>> $O/tune.err
done
for r in 1 2; do
  RAFIKI_TUNE_CACHE=$PWD/$O/db.json timeout -k 10 300 python scripts/bench_pg_gan.py --lods 3,0 --steps 20 --warmup 3 > $O/a$r.json 2>/dev/null
  mv /tmp/shipped_seed_rt/*.json rafiki_amd/tune/
  RAFIKI_TUNE_CACHE=off timeout -k 10 300 python scripts/bench_pg_gan.py --lods 3,0 --steps 20 --warmup 3 > $O/b$r.json 2>/dev/null
  mv rafiki_amd/tune/*.json /tmp/shipped_seed_rt/
done
mv /tmp/shipped_seed_rt/*.json rafiki_amd/tune/
for f in a1 b1 a2 b2; do python3 -c "
import json
d = json.loads([l for l in open('$O/$f.json') if l.startswith('{')][-1])
print('$f', ' '.join('lod%s %.3f' % (k, v['ms_per_round']) for k, v in d['lods'].items()))"; done > $O/ab.txt
cat $O/ab.txt
python3 - <<'PY'
import glob, json
new = json.load(open('gpurun_out/rt/db.json'))
old = json.load(open(glob.glob('rafiki_amd/tune/*.json')[0]))
for k in sorted(set(new) - set(k for k in old if k in new and old[k] == new[k])):
    if json.loads(k)[0] == 'sw':
        print(k, 'shipped', old.get(k), 'retuned', new[k])
PY
