"""Dataset converters (reference examples/datasets/*) on synthetic inputs of the real formats."""
import os
import zipfile

import numpy as np

from rafiki_amd import datasets as DS
from rafiki_amd.model import dataset_utils
from rafiki_amd.model.tfrecord import TFRecordImageDataset


def test_mnist_idx_to_image_files(tmp_path):
    rng = np.random.RandomState(0)
    x = rng.randint(0, 256, (30, 28, 28)).astype(np.uint8)
    y = (np.arange(30) % 4).astype(np.uint8)
    p = {k: str(tmp_path / k) for k in ('xi', 'yi', 'xt', 'yt')}
    DS.write_idx(p['xi'], x)
    DS.write_idx(p['yi'], y)
    DS.write_idx(p['xt'], x[:10], compress=False)
    DS.write_idx(p['yt'], y[:10], compress=False)
    assert (DS.read_idx(p['xi']) == x).all() and (DS.read_idx(p['yt']) == y[:10]).all()
    tr, te, meta = DS.load_mnist_format(p['xi'], p['yi'], p['xt'], p['yt'], {0: 'a', 1: 'b', 2: 'c', 3: 'd'},
                                        str(tmp_path / 'tr.zip'), str(tmp_path / 'te.zip'),
                                        str(tmp_path / 'meta.csv'), limit=20)
    ds = dataset_utils.load_dataset_of_image_files(tr)
    imgs, labels = ds.as_arrays()
    assert len(labels) == 20 and ds.classes == 4
    order = np.argsort([int(n.split('-')[1].split('.')[0]) for n in
                        [r for r in zipfile.ZipFile(tr).namelist() if r.endswith('.png')]])
    assert sorted(labels.tolist()) == sorted(y[:20].tolist())
    assert open(meta).read().splitlines()[1] == '0,a'


def test_ptb_to_corpus(tmp_path):
    src = tmp_path / 'treebank.zip'
    with zipfile.ZipFile(src, 'w') as zf:
        zf.writestr('treebank/tagged/wsj_0001.pos', '\n======\n\n[ Pierre/NNP Vinken/NNP ]\n,/, 61/CD years/NNS\n\n'
                                                    '======\n\nMr./NNP Vinken/NNP is/VBZ chairman/NN ./.\n')
        for i in range(2, 21):
            zf.writestr('treebank/tagged/wsj_%04d.pos' % i, 'The/DT cat/NN sat/VBD ./.\n')
    tr, te, meta = DS.load_ptb_format(str(src), str(tmp_path / 'tr.zip'), str(tmp_path / 'te.zip'),
                                      str(tmp_path / 'meta.tsv'))
    c = dataset_utils.load_dataset_of_corpus(tr)
    assert c.size == 2 + 18 and c[0][0][0] == 'Pierre' and len(c[0]) == 5 and len(c[1]) == 5
    assert dataset_utils.load_dataset_of_corpus(te).size == 1
    tags = [l.split('\t')[1] for l in open(meta).read().splitlines()[1:]]
    assert tags[:3] == ['NNP', ',', 'CD']


def test_image_generation_converters(tmp_path):
    rng = np.random.RandomState(1)
    x = rng.randint(0, 256, (12, 28, 28)).astype(np.uint8)
    DS.write_idx(str(tmp_path / 'x'), x)
    DS.write_idx(str(tmp_path / 'y'), (np.arange(12) % 10).astype(np.uint8))
    d = DS.load_mnist_tfrecords(str(tmp_path / 'x'), str(tmp_path / 'y'), str(tmp_path / 'mnist'))
    ds = TFRecordImageDataset(d)
    assert ds.shape == [1, 32, 32] and ds.images[0][:, :, 2:30, 2:30].sum() > 0 and ds.label_size == 10
    assert ds.images[0][:, :, :2].sum() == 0  # zero padding
    # CIFAR-10 binary batches
    cdir = tmp_path / 'cifar'
    cdir.mkdir()
    for b in (1, 2):
        recs = np.concatenate([np.full((5, 1), b, np.uint8), rng.randint(0, 256, (5, 3072)).astype(np.uint8)], 1)
        recs.tofile(str(cdir / 'data_batch_{}.bin'.format(b)))
    ds = TFRecordImageDataset(DS.load_cifar_tfrecords(str(cdir), str(tmp_path / 'c10')))
    assert ds.shape == [3, 32, 32] and ds.num_images == 10
    # user images (non power of two -> resized down)
    from PIL import Image
    udir = tmp_path / 'user'
    udir.mkdir()
    for i in range(3):
        Image.fromarray(rng.randint(0, 256, (40, 40, 3)).astype(np.uint8)).save(str(udir / '{}.png'.format(i)))
    ds = TFRecordImageDataset(DS.load_user_dataset(str(udir), str(tmp_path / 'u')))
    assert ds.shape == [3, 32, 32] and ds.num_images == 3
