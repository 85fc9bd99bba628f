"""Dataset converters: produce the dataset types Rafiki tasks consume (reference
examples/datasets/*).

* ``load_mnist_format`` — MNIST-format IDX files -> IMAGE_FILES zips + meta CSV
  (reference image_classification/load_mnist_format.py:15-98);
* ``load_ptb_format`` — Penn-Treebank-sample ``treebank/tagged/*.pos`` -> CORPUS zips + meta TSV
  (reference pos_tagging/load_ptb_format.py:15-150);
* ``load_mnist_tfrecords`` / ``load_cifar_tfrecords`` / ``load_user_dataset`` — IMAGE_GENERATION
  TFRecord directories (reference image_generation/load_mnist.py:85-116, load_cifar10.py,
  load_cifar100.py, load_user_dataset.py).

Inputs are local paths or ``file://`` URIs (``dataset_utils.download_dataset_from_uri`` also
accepts http(s) where a network exists).  CIFAR is read from the binary distribution
(``data_batch_*.bin`` / ``train.bin``: raw bytes) rather than the pickled python one, so no pickle
is ever loaded from a dataset file.
"""
from __future__ import annotations

import csv
import glob
import gzip
import io
import os
import re
import shutil
import tempfile
import zipfile
from itertools import chain
from typing import Dict, Optional

import numpy as np

from ..model import dataset_utils
from ..model.tfrecord import write_tfrecord_dataset


# ------------------------------------------------------------------------- IMAGE_FILES (MNIST)
def read_idx(path: str) -> np.ndarray:
    """IDX (gzip or raw) -> ndarray; dims from the header (http://yann.lecun.com/exdb/mnist/)."""
    opener = gzip.open if _is_gzip(path) else open
    with opener(path, 'rb') as f:
        data = f.read()
    if data[0] != 0 or data[1] != 0:
        raise ValueError('not an IDX file: {}'.format(path))
    dtype = {0x08: np.uint8, 0x09: np.int8, 0x0B: '>i2', 0x0C: '>i4', 0x0D: '>f4', 0x0E: '>f8'}[data[2]]
    nd = data[3]
    dims = [int.from_bytes(data[4 + 4 * i:8 + 4 * i], 'big') for i in range(nd)]
    return np.frombuffer(data, dtype=dtype, offset=4 + 4 * nd).reshape(dims)


def write_idx(path: str, arr: np.ndarray, compress: bool = True):
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    head = bytes([0, 0, 0x08, arr.ndim]) + b''.join(int(d).to_bytes(4, 'big') for d in arr.shape)
    opener = gzip.open if compress else open
    with opener(path, 'wb') as f:
        f.write(head + arr.tobytes())
    return path


def _is_gzip(path):
    with open(path, 'rb') as f:
        return f.read(2) == b'\x1f\x8b'


def load_mnist_format(train_images_url, train_labels_url, test_images_url, test_labels_url,
                      label_to_name: Dict[int, str], out_train_dataset_path, out_test_dataset_path,
                      out_meta_csv_path, limit: Optional[int] = None):
    fetch = dataset_utils.download_dataset_from_uri
    tr_x, tr_y = read_idx(fetch(train_images_url)), read_idx(fetch(train_labels_url))
    te_x, te_y = read_idx(fetch(test_images_url)), read_idx(fetch(test_labels_url))
    if limit is not None:
        tr_x, tr_y, te_x, te_y = tr_x[:limit], tr_y[:limit], te_x[:limit], te_y[:limit]
    label_to_index = {}
    with open(out_meta_csv_path, 'w', newline='') as f:
        w = csv.DictWriter(f, fieldnames=['class', 'name'])
        w.writeheader()
        for i, label in enumerate(sorted(set(int(v) for v in chain(tr_y, te_y)))):
            label_to_index[label] = i
            w.writerow({'class': i, 'name': label_to_name.get(label, str(label))})
    _write_image_files(tr_x, tr_y, label_to_index, out_train_dataset_path)
    _write_image_files(te_x, te_y, label_to_index, out_test_dataset_path)
    return out_train_dataset_path, out_test_dataset_path, out_meta_csv_path


def _write_image_files(images, labels, label_to_index, out_path):
    from PIL import Image
    os.makedirs(os.path.dirname(os.path.abspath(out_path)), exist_ok=True)
    with zipfile.ZipFile(out_path, 'w', zipfile.ZIP_DEFLATED) as zf:
        out = io.StringIO()
        w = csv.DictWriter(out, fieldnames=['path', 'class'])
        w.writeheader()
        for i, (img, label) in enumerate(zip(images, labels)):
            name = '{}-{}.png'.format(int(label), i)
            buf = io.BytesIO()
            Image.fromarray(np.asarray(img, dtype=np.uint8)).save(buf, format='PNG')
            zf.writestr(name, buf.getvalue())
            w.writerow({'path': name, 'class': label_to_index[int(label)]})
        zf.writestr('images.csv', out.getvalue())
    return out_path


# ------------------------------------------------------------------------------ CORPUS (PTB)
_SEP = re.compile(r'^[=\s]+$')
_TOK = re.compile(r'(\S+)/(\S+)')


def _read_sentences(lines, tag_to_index):
    sent, started = [], False
    for line in chain(lines, [None]):
        if line is None or _SEP.match(line):
            if started and sent:
                yield sent
            sent, started = [], False
            continue
        started = True
        for m in _TOK.finditer(line):
            tok, tag = m.group(1), m.group(2)
            if tag not in tag_to_index:
                tag_to_index[tag] = len(tag_to_index)
            sent.append([tok, tag_to_index[tag]])


def load_ptb_format(dataset_url, out_train_dataset_path, out_test_dataset_path, out_meta_tsv_path,
                    test_files_ratio: float = 0.05):
    """PTB sample zip (``treebank/tagged/*.pos``, ``word/TAG`` tokens, sentences separated by blank
    or ``=====`` lines) -> train/test CORPUS zips (``corpus.tsv`` token/tag, ``\\n`` separators)."""
    path = dataset_utils.download_dataset_from_uri(dataset_url)
    tag_to_index: Dict[str, int] = {}
    with tempfile.TemporaryDirectory() as d:
        with zipfile.ZipFile(path) as zf:
            zf.extractall(d)
        files = sorted(glob.glob(os.path.join(d, 'treebank', 'tagged', '*.pos')))
        if not files:
            raise ValueError('no treebank/tagged/*.pos files in {}'.format(dataset_url))
        n_train = int(round(len(files) * (1 - test_files_ratio)))
        parts = {'train': files[:n_train], 'test': files[n_train:]}
        sents = {}
        for k, fs in parts.items():
            sents[k] = []
            for p in fs:
                with open(p, errors='replace') as f:
                    sents[k].extend(_read_sentences(f, tag_to_index))
    from ..model.dataset import write_corpus_zip
    write_corpus_zip(out_train_dataset_path, sents['train'])
    write_corpus_zip(out_test_dataset_path, sents['test'])
    index_to_tag = {v: k for k, v in tag_to_index.items()}
    with open(out_meta_tsv_path, 'w') as f:
        f.write('tag\tname\n')
        for i in range(len(index_to_tag)):
            f.write('{}\t{}\n'.format(i, index_to_tag[i]))
    return out_train_dataset_path, out_test_dataset_path, out_meta_tsv_path


# ------------------------------------------------------------------ IMAGE_GENERATION (TFRecords)
def load_mnist_tfrecords(train_images_url, train_labels_url, out_train_dataset_path, pad_to: int = 32):
    """MNIST IDX -> TFRecord dir, 28x28 zero-padded to 32x32, one-hot labels (load_mnist.py:94-114)."""
    fetch = dataset_utils.download_dataset_from_uri
    images = read_idx(fetch(train_images_url)).reshape(-1, 1, 28, 28)
    labels = read_idx(fetch(train_labels_url)).astype(np.int64)
    p = (pad_to - 28) // 2
    images = np.pad(images, [(0, 0), (0, 0), (p, p), (p, p)], 'constant', constant_values=0)
    return write_tfrecord_dataset(out_train_dataset_path, images, labels)


def read_cifar_bin(paths, label_bytes=1, label_index=0) -> tuple:
    """CIFAR binary batches: records of ``label_bytes`` label byte(s) + 3072 image bytes (CHW).
    CIFAR-100 has 2 label bytes (coarse, fine): label_index=1 picks fine."""
    rec = label_bytes + 3072
    xs, ys = [], []
    for p in paths:
        raw = np.fromfile(p, dtype=np.uint8)
        raw = raw[:raw.size // rec * rec].reshape(-1, rec)
        ys.append(raw[:, label_index].astype(np.int64))
        xs.append(raw[:, label_bytes:].reshape(-1, 3, 32, 32))
    return np.concatenate(xs), np.concatenate(ys)


def load_cifar_tfrecords(bin_dir, out_train_dataset_path, cifar100: bool = False):
    """CIFAR-10 (``data_batch_1..5.bin``) or CIFAR-100 (``train.bin``, fine labels) -> TFRecord dir."""
    if cifar100:
        x, y = read_cifar_bin([os.path.join(bin_dir, 'train.bin')], label_bytes=2, label_index=1)
    else:
        x, y = read_cifar_bin(sorted(glob.glob(os.path.join(bin_dir, 'data_batch_*.bin'))))
    if len(x) == 0:
        raise ValueError('no CIFAR binary batches under {}'.format(bin_dir))
    return write_tfrecord_dataset(out_train_dataset_path, x, y)


def load_user_dataset(train_dataset_path, out_train_dataset_path):
    """A directory of same-size square RGB/grayscale images -> TFRecord dir, resized down to a power
    of two when needed (load_user_dataset.py:9-44)."""
    from PIL import Image
    files = sorted(f for f in glob.glob(os.path.join(train_dataset_path, '*')) if os.path.isfile(f))
    if not files:
        raise ValueError('no input images in {}'.format(train_dataset_path))
    first = np.asarray(Image.open(files[0]))
    res = first.shape[0]
    if first.shape[1] != res:
        raise ValueError('input images must be square')
    ch = first.shape[2] if first.ndim == 3 else 1
    if ch not in (1, 3):
        raise ValueError('input images must be RGB or grayscale')
    target = 2 ** int(np.floor(np.log2(res)))
    imgs = []
    for p in files:
        im = Image.open(p)
        if target != res:
            im = im.resize((target, target), Image.LANCZOS)
        a = np.asarray(im)
        imgs.append(a[None] if ch == 1 else a.transpose(2, 0, 1))
    return write_tfrecord_dataset(out_train_dataset_path, np.stack(imgs))


def copy_dataset(src, dst):
    shutil.copyfile(src, dst)
    return dst
