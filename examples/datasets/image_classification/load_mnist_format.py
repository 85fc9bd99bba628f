"""Convert MNIST-format IDX files (e.g. Fashion-MNIST) to IMAGE_FILES zips + meta CSV.

usage: python load_mnist_format.py <train-images> <train-labels> <test-images> <test-labels> [--limit N]
(local paths or URLs; reference examples/datasets/image_classification/load_mnist_format.py)"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', '..'))
from rafiki_amd.datasets import load_mnist_format  # noqa: E402

FASHION = {0: 'T-shirt/top', 1: 'Trouser', 2: 'Pullover', 3: 'Dress', 4: 'Coat', 5: 'Sandal', 6: 'Shirt',
           7: 'Sneaker', 8: 'Bag', 9: 'Ankle boot'}

if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    for k in ('train_images', 'train_labels', 'test_images', 'test_labels'):
        ap.add_argument(k)
    ap.add_argument('--limit', type=int, default=None)
    ap.add_argument('--out_dir', default='data')
    a = ap.parse_args()
    os.makedirs(a.out_dir, exist_ok=True)
    out = load_mnist_format(a.train_images, a.train_labels, a.test_images, a.test_labels, FASHION,
                            os.path.join(a.out_dir, 'fashion_mnist_for_image_classification_train.zip'),
                            os.path.join(a.out_dir, 'fashion_mnist_for_image_classification_test.zip'),
                            os.path.join(a.out_dir, 'fashion_mnist_for_image_classification_meta.csv'), a.limit)
    print('\n'.join(out))
