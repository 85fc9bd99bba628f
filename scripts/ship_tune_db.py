"""Install a node-wide autotune database captured on an MI355X as the package's read-only seed
(rafiki_amd/tune/<arch>-<kernel library hash>.json), replacing seeds of older kernel builds.

usage: python scripts/ship_tune_db.py <captured.json> [--arch gfx950]
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
    ap.add_argument('db')
    ap.add_argument('--arch', default='gfx950')
    a = ap.parse_args()
    from rafiki_amd.ops import autotune
    autotune._ident['arch'] = a.arch
    with open(a.db) as f:
        entries = json.load(f)
    dst_dir = autotune.SHIPPED_DIR
    os.makedirs(dst_dir, exist_ok=True)
    for old in glob.glob(os.path.join(dst_dir, a.arch + '-*.json')):
        os.remove(old)
    dst = os.path.join(dst_dir, autotune.db_name())
    with open(dst, 'w') as f:
        json.dump(entries, f, sort_keys=True, indent=0)
    print('shipped {} entries -> {}'.format(len(entries), dst))


if __name__ == '__main__':
    main()
