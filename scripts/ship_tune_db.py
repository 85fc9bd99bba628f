"""Install a node-wide autotune database captured on an MI355X as the package's read-only seed
(rafiki_amd/tune/<arch>-<kernel library hash>.json), replacing seeds of older kernel builds.

usage: python scripts/ship_tune_db.py <captured.json> [--arch gfx950] [--merge]
       python scripts/ship_tune_db.py --rekey     (sources changed where no pick depends on them: keep
                                                   the shipped picks under the new source hash)
The captured file must come from a run of THIS kernel library (same librafiki_kernels.so bytes): the
seed is keyed by its content hash, so a rebuilt library simply ignores it.
"""
import argparse
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db', nargs='?')
    ap.add_argument('--arch', default='gfx950')
    ap.add_argument('--merge', action='store_true', help='keep shipped entries the captured file lacks')
    ap.add_argument('--rekey', action='store_true')
    a = ap.parse_args()
    from rafiki_amd.ops import autotune
    autotune._ident['arch'] = a.arch
    dst_dir = autotune.SHIPPED_DIR
    olds = sorted(glob.glob(os.path.join(dst_dir, a.arch + '-*.json')))
    entries = {}
    if a.rekey or a.merge:
        for old in olds:
            with open(old) as f:
                entries.update(json.load(f))
    if a.db:
        with open(a.db) as f:
            entries.update(json.load(f))
    os.makedirs(dst_dir, exist_ok=True)
    for old in olds:
        os.remove(old)
    dst = os.path.join(dst_dir, autotune.db_name())
    with open(dst, 'w') as f:
        json.dump(entries, f, sort_keys=True, indent=0)
    print('shipped {} entries -> {}'.format(len(entries), dst))


if __name__ == '__main__':
    main()
