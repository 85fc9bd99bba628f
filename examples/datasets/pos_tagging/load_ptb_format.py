"""Convert a Penn-Treebank-sample zip (treebank/tagged/*.pos) to CORPUS zips + meta TSV.

usage: python load_ptb_format.py <treebank.zip> [--out_dir data]
(reference examples/datasets/pos_tagging/load_ptb_format.py)"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', '..'))
from rafiki_amd.datasets import load_ptb_format  # noqa: E402

if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('dataset')
    ap.add_argument('--out_dir', default='data')
    a = ap.parse_args()
    os.makedirs(a.out_dir, exist_ok=True)
    print('\n'.join(load_ptb_format(a.dataset, os.path.join(a.out_dir, 'ptb_for_pos_tagging_train.zip'),
                                    os.path.join(a.out_dir, 'ptb_for_pos_tagging_test.zip'),
                                    os.path.join(a.out_dir, 'ptb_for_pos_tagging_meta.tsv'))))
