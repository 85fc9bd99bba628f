"""Build an IMAGE_GENERATION TFRecord directory (multi-resolution, reference format).

usage:
  python load_dataset.py mnist <train-images-idx> <train-labels-idx> [--out data/mnist_for_image_generation]
  python load_dataset.py cifar10 <dir with data_batch_*.bin> [--out ...]
  python load_dataset.py cifar100 <dir with train.bin> [--out ...]
  python load_dataset.py user <dir of square images> [--out ...]
(reference examples/datasets/image_generation/load_{mnist,cifar10,cifar100,user_dataset}.py)"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', '..'))
from rafiki_amd import datasets as DS  # noqa: E402

if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('kind', choices=['mnist', 'cifar10', 'cifar100', 'user'])
    ap.add_argument('inputs', nargs='+')
    ap.add_argument('--out', default=None)
    a = ap.parse_args()
    out = a.out or os.path.join('data', '{}_for_image_generation'.format(a.kind))
    if a.kind == 'mnist':
        print(DS.load_mnist_tfrecords(a.inputs[0], a.inputs[1], out))
    elif a.kind in ('cifar10', 'cifar100'):
        print(DS.load_cifar_tfrecords(a.inputs[0], out, cifar100=a.kind == 'cifar100'))
    else:
        print(DS.load_user_dataset(a.inputs[0], out))
