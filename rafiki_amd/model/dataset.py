"""Dataset loading for models (reference rafiki/model/dataset.py:25-270, redesigned).

Formats (docs/src/user/datasets.rst:18-85 of the reference):
  * IMAGE_FILES : zip with ``images.csv`` (``path,class``) + image files
  * CORPUS      : zip with ``corpus.tsv`` (``token`` + tag columns, sentences split by a ``\\n`` token)

Design changes for one MI355X node:
  * images are decoded ONCE, eagerly and in parallel, into one contiguous uint8 array, so a model
    can upload the whole split to HBM (288 GB/GPU) and do all shuffling/batching on the device;
  * ``synthetic://`` URIs generate deterministic datasets of a given shape in memory — there is no
    network on the target, so benchmarks and tests use these (documented as synthetic data);
  * ``classes`` is ``max(label) + 1`` rather than the number of distinct labels of the split
    (reference bug (j), dataset.py:265).
"""
from __future__ import annotations

import collections
import csv
import io
import os
import tempfile
import threading
import zipfile
from concurrent.futures import ThreadPoolExecutor
from urllib.parse import parse_qs, urlparse

import numpy as np

from ..constants import DatasetType  # noqa: F401  (re-exported for model code)


class InvalidDatasetProtocolException(Exception):
    pass


class InvalidDatasetTypeException(Exception):
    pass


class InvalidDatasetFormatException(Exception):
    pass


class ModelDataset:
    def __init__(self, dataset_path):
        self.path = dataset_path
        self.size = 0

    def __getitem__(self, index):
        raise NotImplementedError()

    def __len__(self):
        return self.size


class ImageFilesDataset(ModelDataset):
    """(image uint8 [H, W] or [H, W, C], class int) samples, all decoded into ``self.images``."""

    def __init__(self, dataset_path, image_size=None, images=None, labels=None):
        super().__init__(dataset_path)
        self.image_size = image_size
        if images is None:
            images, labels = self._load_zip(dataset_path, image_size)
        self.images = np.ascontiguousarray(images)
        self.labels = np.asarray(labels, dtype=np.int64)
        self.size = len(self.labels)
        self.classes = int(self.labels.max()) + 1 if self.size else 0

    def __getitem__(self, index):
        return self.images[index], int(self.labels[index])

    def as_arrays(self):
        return self.images, self.labels

    @staticmethod
    def _load_zip(path, image_size):
        from PIL import Image
        with zipfile.ZipFile(path, 'r') as zf:
            try:
                rows = list(csv.DictReader(io.TextIOWrapper(zf.open('images.csv'), 'utf-8')))
                paths = [r['path'] for r in rows]
                labels = [int(r['class']) for r in rows]
            except Exception as e:
                raise InvalidDatasetFormatException(str(e))
            blobs = [zf.read(p) for p in paths]

        def decode(b):
            im = Image.open(io.BytesIO(b))
            if image_size is not None:
                size = (image_size, image_size) if isinstance(image_size, int) else tuple(image_size)
                im = im.resize(size)
            return np.asarray(im, dtype=np.uint8)

        workers = min(16, os.cpu_count() or 4)
        with ThreadPoolExecutor(workers) as ex:
            images = list(ex.map(decode, blobs, chunksize=256))
        if not images:
            return np.zeros((0, 1, 1), np.uint8), labels
        return np.stack(images), labels


class CorpusDataset(ModelDataset):
    """Sentences of ``[token, tag_1, ..., tag_k]`` rows."""

    def __init__(self, dataset_path, tags=('tag',), split_by='\\n', sents=None):
        super().__init__(dataset_path)
        self.tags = list(tags)
        if sents is None:
            sents = self._load_zip(dataset_path, self.tags, split_by)
        self._sents = sents
        self.size = len(sents)
        self.tag_num_classes = [0] * len(self.tags)
        self.max_token_len = 0
        self.max_sent_len = 0
        for s in sents:
            self.max_sent_len = max(self.max_sent_len, len(s))
            for tok in s:
                self.max_token_len = max(self.max_token_len, len(tok[0]))
                for i, t in enumerate(tok[1:]):
                    self.tag_num_classes[i] = max(self.tag_num_classes[i], t + 1)

    def __getitem__(self, index):
        return self._sents[index]

    @staticmethod
    def _load_zip(path, tags, split_by):
        sents, sent = [], []
        with zipfile.ZipFile(path, 'r') as zf:
            try:
                reader = csv.DictReader(io.TextIOWrapper(zf.open('corpus.tsv'), 'utf-8'), dialect='excel-tab')
                for row in reader:
                    token = row.pop('token')
                    if token == split_by:
                        sents.append(sent)
                        sent = []
                        continue
                    sent.append([token, *[int(row[t]) for t in tags]])
            except Exception as e:
                raise InvalidDatasetFormatException(str(e))
        if sent:
            sents.append(sent)
        return sents


# ------------------------------------------------------------------------------- synthetic data
_BANKS = {}
_BANK_BYTES = 256 << 20   # host bytes of the shared noise bank at most (default bank size)


def _noise_bank(shape, nb):
    """The unit-variance Gaussian noise bank of ``synthetic_images``: one fixed bank per image shape,
    SHARED by every split and seed (so train and test noise come from the same distribution) and at
    least as large as the image dimension (so the noise spans the full pixel space)."""
    key = (tuple(shape), nb)
    if key not in _BANKS:
        _BANKS.clear()   # one resident bank (~50 MB for 4096 CIFAR-sized images)
        _BANKS[key] = np.random.default_rng(4321).standard_normal(size=(nb, *shape), dtype=np.float32)
    return _BANKS[key]


def synthetic_images(n, size=32, channels=3, classes=10, seed=0, separable=True, noise=None, flip=0.0,
                     chunk=4096, bank=None):
    """Deterministic class-conditional images: a per-class template plus Gaussian noise (std ``noise``,
    default 48 / 96 for separable / not).  ``flip`` relabels that fraction of the images uniformly at
    random, so no classifier exceeds ~1 - flip*(1 - 1/classes) accuracy (a non-separable task).

    The noise of image i is std * (cos(t_i) B[j_i] + sin(t_i) B[k_i]) over a bank B of ``bank`` unit
    Gaussian images (random pair, random angle: exactly N(0, std^2) per pixel), built chunk by chunk in
    float32 — a CIFAR-sized split (50k x 32x32x3) takes a fraction of a second instead of drawing 150M
    normals, which dominated a benchmark trial's first dataset load.  The bank is shared by all splits
    and seeds and has at least as many images as pixels (default max(4096, dim)), so every split's noise
    has the same full-rank distribution (above 8192 values per image, e.g. 64x64x3, the bank is capped at
    256 MB of host memory, so its rank is the bank size); the seed picks the labels, pairs and angles.  (Round 3 drew a
    1024-image bank per seed — a rank-1024 noise subspace that differed between train and test — so
    scores on this data are not comparable with that round's.)"""
    rng = np.random.default_rng(seed)
    shape = (size, size) if channels == 1 else (size, size, channels)
    tmpl_rng = np.random.default_rng(1234)
    templates = tmpl_rng.uniform(0, 255, size=(classes, *shape)).astype(np.float32)
    templates = templates * np.float32(0.6) + np.float32(50.0)
    labels = rng.integers(0, classes, size=n)
    std = np.float32(noise if noise is not None else (48.0 if separable else 96.0))
    dim = int(np.prod(shape))
    # full rank (>= dim images) while that fits the byte budget; large images cap the bank instead of
    # growing it with the square of the pixel count (128x128x3 would need ~9.7 GB at full rank)
    nb = int(bank) if bank is not None else max(1024, min(max(4096, dim), _BANK_BYTES // (4 * dim)))
    B = _noise_bank(shape, nb)
    j1, j2 = rng.integers(0, nb, size=n), rng.integers(0, nb, size=n)
    th = rng.uniform(0.0, 2.0 * np.pi, size=n)
    ca = (std * np.cos(th)).astype(np.float32).reshape((n,) + (1,) * len(shape))
    sa = (std * np.sin(th)).astype(np.float32).reshape((n,) + (1,) * len(shape))
    imgs = np.empty((n, *shape), dtype=np.uint8)
    for i in range(0, n, chunk):
        sl = slice(i, i + chunk)
        nz = B[j1[sl]] * ca[sl]
        nz += B[j2[sl]] * sa[sl]
        nz += templates[labels[sl]]
        np.clip(nz, 0, 255, out=nz)
        imgs[sl] = nz
    if flip > 0:
        sel = rng.random(n) < float(flip)
        labels = labels.copy()
        labels[sel] = rng.integers(0, classes, size=int(sel.sum()))
    return imgs, labels.astype(np.int64)


def synthetic_corpus(n_sents, vocab=500, tags=12, seed=0, max_len=30):
    rng = np.random.default_rng(seed)
    tag_of_word = np.random.default_rng(99).integers(0, tags, size=vocab)
    sents = []
    for _ in range(n_sents):
        L = int(rng.integers(3, max_len + 1))
        words = rng.integers(0, vocab, size=L)
        sents.append([['w{}'.format(w), int(tag_of_word[w])] for w in words])
    return sents


def _parse_synthetic(uri):
    u = urlparse(uri)
    q = {k: v[0] for k, v in parse_qs(u.query).items()}
    kind = (u.netloc or u.path.strip('/')).lower()
    return kind, q


class ModelDatasetUtils:
    """Global ``dataset_utils`` helper used by models."""

    def __init__(self):
        self._uri_to_path = {}
        # decoded IMAGE_FILES datasets, reused by every trial of a worker process (a train job runs
        # many trials on the same URIs; the reference memoised only the download).  Arrays are
        # handed out read-only; byte budget RAFIKI_DATASET_CACHE_MB (0 disables).
        self._decoded = collections.OrderedDict()
        self._decoded_bytes = 0
        self._lock = threading.Lock()

    def _cache_key(self, dataset_uri, image_size):
        uri = str(dataset_uri)
        if not uri.startswith('synthetic://') and os.path.exists(uri):
            st = os.stat(uri)
            return (uri, image_size, st.st_mtime_ns, st.st_size)
        return (uri, image_size)

    def load_dataset_of_image_files(self, dataset_uri, image_size=None):
        budget = int(os.environ.get('RAFIKI_DATASET_CACHE_MB', '8192')) << 20
        key = self._cache_key(dataset_uri, image_size if image_size is None or isinstance(image_size, int)
                              else tuple(image_size))
        with self._lock:
            hit = self._decoded.get(key)
            if hit is not None:
                self._decoded.move_to_end(key)
                return ImageFilesDataset(dataset_uri, image_size, images=hit[0], labels=hit[1])
        ds = self._load_image_files(dataset_uri, image_size)
        nbytes = ds.images.nbytes + ds.labels.nbytes
        if budget > 0 and nbytes <= budget:
            ds.images.setflags(write=False)
            ds.labels.setflags(write=False)
            with self._lock:
                if key not in self._decoded:
                    self._decoded[key] = (ds.images, ds.labels)
                    self._decoded_bytes += nbytes
                while self._decoded_bytes > budget and self._decoded:
                    _, (im, lb) = self._decoded.popitem(last=False)
                    self._decoded_bytes -= im.nbytes + lb.nbytes
        return ds

    def clear_cache(self):
        with self._lock:
            self._decoded.clear()
            self._decoded_bytes = 0

    def _load_image_files(self, dataset_uri, image_size=None):
        if str(dataset_uri).startswith('synthetic://'):
            kind, q = _parse_synthetic(dataset_uri)
            size = int(q.get('size', image_size or 32))
            imgs, labels = synthetic_images(int(q.get('n', 1024)), size=size, channels=int(q.get('channels', 1)),
                                            classes=int(q.get('classes', 10)), seed=int(q.get('seed', 0)),
                                            noise=float(q['noise']) if 'noise' in q else None,
                                            flip=float(q.get('flip', 0.0)))
            if image_size is not None:  # same contract as a zip: decoded images come back at image_size
                want = (image_size, image_size) if isinstance(image_size, int) else tuple(image_size)
                if imgs.shape[1:3] != tuple(want):
                    imgs = self.resize_as_images(imgs, want)
            return ImageFilesDataset(dataset_uri, image_size, images=imgs, labels=labels)
        return ImageFilesDataset(self.download_dataset_from_uri(dataset_uri), image_size)

    def load_dataset_of_corpus(self, dataset_uri, tags=('tag',), split_by='\\n'):
        if str(dataset_uri).startswith('synthetic://'):
            _, q = _parse_synthetic(dataset_uri)
            sents = synthetic_corpus(int(q.get('n', 200)), vocab=int(q.get('vocab', 500)),
                                     tags=int(q.get('tags', 12)), seed=int(q.get('seed', 0)))
            return CorpusDataset(dataset_uri, tags, split_by, sents=sents)
        return CorpusDataset(self.download_dataset_from_uri(dataset_uri), tags, split_by)

    def resize_as_images(self, images, image_size):
        from PIL import Image
        size = (image_size, image_size) if isinstance(image_size, int) else tuple(image_size)
        return np.asarray([np.asarray(Image.fromarray(np.asarray(x, dtype=np.uint8)).resize(size)) for x in images])

    def download_dataset_from_uri(self, dataset_uri):
        if dataset_uri in self._uri_to_path:
            return self._uri_to_path[dataset_uri]
        u = urlparse(dataset_uri)
        proto = (u.scheme or '').lower()
        if proto in ('http', 'https'):
            import requests
            r = requests.get(dataset_uri, stream=True, timeout=60)
            r.raise_for_status()
            f = tempfile.NamedTemporaryFile(delete=False)
            for chunk in r.iter_content(1 << 20):
                f.write(chunk)
            f.close()
            path = f.name
        elif proto in ('', 'file'):
            path = u.path if proto == 'file' else dataset_uri
        else:
            raise InvalidDatasetProtocolException(proto)
        self._uri_to_path[dataset_uri] = path
        return path


def write_image_files_zip(path, images, labels, fmt='png'):
    """Write an IMAGE_FILES dataset zip (what examples/datasets converters produce)."""
    from PIL import Image
    with zipfile.ZipFile(path, 'w', compression=zipfile.ZIP_STORED) as zf:
        lines = ['path,class']
        for i, (im, y) in enumerate(zip(images, labels)):
            name = 'images/{}.{}'.format(i, fmt)
            buf = io.BytesIO()
            Image.fromarray(np.asarray(im, dtype=np.uint8)).save(buf, format=fmt.upper())
            zf.writestr(name, buf.getvalue())
            lines.append('{},{}'.format(name, int(y)))
        zf.writestr('images.csv', '\n'.join(lines) + '\n')
    return path


def write_corpus_zip(path, sents, tags=('tag',), split_by='\\n'):
    with zipfile.ZipFile(path, 'w') as zf:
        out = io.StringIO()
        w = csv.writer(out, dialect='excel-tab')
        w.writerow(['token', *tags])
        for s in sents:
            for tok in s:
                w.writerow(tok)
            w.writerow([split_by, *([0] * len(tags))])
        zf.writestr('corpus.tsv', out.getvalue())
    return path


dataset_utils = ModelDatasetUtils()
