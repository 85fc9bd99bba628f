"""TFRecord multi-resolution image datasets without TensorFlow.

The reference's IMAGE_GENERATION datasets are directories of ``<name>-rNN.tfrecords`` files (one
per level of detail, NN = log2 resolution) holding ``tf.train.Example`` records with features
``shape`` (int64 [C, H, W]) and ``data`` (raw uint8 bytes), plus an optional ``*-rxx.labels`` numpy
file (pg_gans.py:380-597).  This module reads and writes exactly that format:

* record framing: ``u64 length | u32 masked-crc32c(length) | payload | u32 masked-crc32c(payload)``;
* payload: the protobuf wire encoding of Example{Features{map<string, Feature>}} — encoded and
  decoded by hand (no generated proto classes needed);
* ``TFRecordExporter`` mirrors the reference exporter (2x2 box-filter pyramid, rint/clip to uint8,
  labels via ``np.save``), so datasets made by either tool are interchangeable.
"""
from __future__ import annotations

import ctypes
import glob
import os
import struct
from typing import Dict, Iterator, List, Optional, Tuple

import numpy as np

# ------------------------------------------------------------------------------------ crc32c
_CRC_TABLE = None


def _table():
    global _CRC_TABLE
    if _CRC_TABLE is None:
        poly = 0x82F63B78
        t = np.zeros(256, dtype=np.uint32)
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ poly if c & 1 else c >> 1
            t[i] = c
        _CRC_TABLE = [int(v) for v in t]
    return _CRC_TABLE


def crc32c(data: bytes) -> int:
    from .. import runtime
    h = runtime.lib()
    if h is not None:
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        return int(h.rt_crc32c(buf, len(data)))
    t = _table()
    c = 0xFFFFFFFF
    for b in data:
        c = t[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ------------------------------------------------------------------------------- record I/O
def iter_records(path: str, verify: bool = False) -> Iterator[bytes]:
    with open(path, 'rb') as f:
        while True:
            head = f.read(12)
            if not head:
                return
            if len(head) < 12:
                raise ValueError('truncated TFRecord header in {}'.format(path))
            (n,) = struct.unpack('<Q', head[:8])
            if verify and struct.unpack('<I', head[8:])[0] != masked_crc(head[:8]):
                raise ValueError('bad length crc in {}'.format(path))
            payload = f.read(n)
            tail = f.read(4)
            if len(payload) < n or len(tail) < 4:
                raise ValueError('truncated TFRecord in {}'.format(path))
            if verify and struct.unpack('<I', tail)[0] != masked_crc(payload):
                raise ValueError('bad payload crc in {}'.format(path))
            yield payload


class RecordWriter:
    def __init__(self, path: str):
        self.f = open(path, 'wb')

    def write(self, payload: bytes):
        head = struct.pack('<Q', len(payload))
        self.f.write(head + struct.pack('<I', masked_crc(head)) + payload + struct.pack('<I', masked_crc(payload)))

    def close(self):
        self.f.close()


# ------------------------------------------------------------------------- protobuf (Example)
def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf: bytes, i: int) -> Tuple[int, int]:
    shift = v = 0
    while True:
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, i
        shift += 7


def _ld(field: int, payload: bytes) -> bytes:
    return _varint((field << 3) | 2) + _varint(len(payload)) + payload


def _fields(buf: bytes):
    i = 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        field, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(buf, i)
        elif wt == 2:
            n, i = _read_varint(buf, i)
            v = buf[i:i + n]
            i += n
        elif wt == 5:
            v = buf[i:i + 4]
            i += 4
        elif wt == 1:
            v = buf[i:i + 8]
            i += 8
        else:
            raise ValueError('unsupported protobuf wire type {}'.format(wt))
        yield field, wt, v


def encode_example(features: Dict[str, object]) -> bytes:
    """features: name -> bytes | list[int] (int64_list) | list[float] (float_list)."""
    entries = b''
    for name, val in features.items():
        if isinstance(val, (bytes, bytearray)):
            feat = _ld(1, _ld(1, bytes(val)))  # Feature.bytes_list{value}
        elif all(isinstance(x, (int, np.integer)) for x in val):
            feat = _ld(3, _ld(1, b''.join(_varint(int(x)) for x in val)))  # packed int64
        else:
            feat = _ld(2, _ld(1, struct.pack('<{}f'.format(len(val)), *[float(x) for x in val])))
        entries += _ld(1, _ld(1, name.encode()) + _ld(2, feat))
    return _ld(1, entries)  # Example.features


def decode_example(payload: bytes) -> Dict[str, object]:
    out = {}
    for f, wt, features in _fields(payload):
        if f != 1 or wt != 2:
            continue
        for f2, _, entry in _fields(features):
            if f2 != 1:
                continue
            key, feat = None, b''
            for f3, _, v in _fields(entry):
                if f3 == 1:
                    key = bytes(v).decode()
                elif f3 == 2:
                    feat = v
            val = None
            for kind, wt4, lst in _fields(feat):
                if kind == 1:
                    val = [bytes(v) for f5, _, v in _fields(lst) if f5 == 1]
                elif kind == 3:
                    vals = []
                    for f5, wt5, v in _fields(lst):
                        if wt5 == 2:
                            j = 0
                            while j < len(v):
                                x, j = _read_varint(v, j)
                                vals.append(x - (1 << 64) if x >= 1 << 63 else x)
                        else:
                            vals.append(v - (1 << 64) if v >= 1 << 63 else v)
                    val = vals
                elif kind == 2:
                    vals = []
                    for f5, wt5, v in _fields(lst):
                        if wt5 == 2:
                            vals.extend(struct.unpack('<{}f'.format(len(v) // 4), v))
                        else:
                            vals.append(struct.unpack('<f', v)[0])
                    val = vals
            out[key] = val
    return out


def parse_image_record(payload: bytes) -> np.ndarray:
    ex = decode_example(payload)
    shape = [int(s) for s in ex['shape']]
    return np.frombuffer(ex['data'][0], dtype=np.uint8).reshape(shape)


# --------------------------------------------------------------------------------- datasets
def downscale_images(img: np.ndarray) -> np.ndarray:
    """[.., C, H, W] float -> 2x2 box filter (the exporter's pyramid step, pg_gans.py:578-580)."""
    return (img[..., 0::2, 0::2] + img[..., 0::2, 1::2] + img[..., 1::2, 0::2] + img[..., 1::2, 1::2]) * 0.25


class TFRecordExporter:
    """Writes ``<dir>/<basename>-rNN.tfrecords`` for every LOD down to 4x4 (pg_gans.py:529-597)."""

    def __init__(self, tfrecord_dir: str, expected_images: int = 0):
        self.tfrecord_dir = tfrecord_dir
        self.prefix = os.path.join(tfrecord_dir, os.path.basename(os.path.normpath(tfrecord_dir)))
        self.expected_images = expected_images
        self.cur_images = 0
        self.shape = None
        self.writers: List[RecordWriter] = []
        os.makedirs(tfrecord_dir, exist_ok=True)

    def choose_shuffled_order(self):
        order = np.arange(self.expected_images)
        np.random.RandomState(123).shuffle(order)
        return order

    def add_image(self, img: np.ndarray):
        img = np.asarray(img)
        if self.shape is None:
            self.shape = img.shape
            log2 = int(np.log2(self.shape[1]))
            assert self.shape[0] in (1, 3) and self.shape[1] == self.shape[2] == 2 ** log2, self.shape
            for lod in range(log2 - 1):
                self.writers.append(RecordWriter(self.prefix + '-r%02d.tfrecords' % (log2 - lod)))
        assert img.shape == self.shape, (img.shape, self.shape)
        cur = img
        for lod, w in enumerate(self.writers):
            if lod:
                cur = downscale_images(cur.astype(np.float32))
            q = np.rint(cur).clip(0, 255).astype(np.uint8)
            w.write(encode_example({'shape': list(q.shape), 'data': q.tobytes()}))
        self.cur_images += 1

    def add_labels(self, labels: np.ndarray):
        assert labels.shape[0] == self.cur_images
        with open(self.prefix + '-rxx.labels', 'wb') as f:
            np.save(f, labels.astype(np.float32))

    def close(self):
        for w in self.writers:
            w.close()
        self.writers = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def write_tfrecord_dataset(tfrecord_dir: str, images: np.ndarray, labels: Optional[np.ndarray] = None,
                           shuffle: bool = True) -> str:
    """images: uint8 [N, C, H, W] (or [N, H, W] grayscale).  labels: optional [N] ints (one-hot saved)."""
    images = np.asarray(images)
    if images.ndim == 3:
        images = images[:, None]
    with TFRecordExporter(tfrecord_dir, len(images)) as ex:
        order = ex.choose_shuffled_order() if shuffle else np.arange(len(images))
        for i in order:
            ex.add_image(images[i])
        if labels is not None:
            labels = np.asarray(labels)
            if labels.ndim == 1:
                onehot = np.zeros((labels.size, int(labels.max()) + 1), np.float32)
                onehot[np.arange(labels.size), labels] = 1.0
                labels = onehot
            ex.add_labels(labels[order])
    return tfrecord_dir


def _read_images(path: str, max_images: Optional[int] = None) -> np.ndarray:
    """Decode every image record of one file into [N, C, H, W] uint8 (native runtime when built)."""
    from .. import runtime
    h = runtime.lib()
    if h is not None:
        shape = (ctypes.c_longlong * 3)()
        n = int(h.rt_tfrecord_info(path.encode(), 0, shape))
        if n < 0:
            raise ValueError('cannot read TFRecord file {} (error {})'.format(path, n))
        if max_images is not None:
            n = min(n, int(max_images))
        shp = [int(v) for v in shape]
        item = int(np.prod(shp))
        out = np.empty([n] + shp, dtype=np.uint8)
        got = int(h.rt_tfrecord_decode_images(path.encode(), out.ctypes.data, n, item, 0))
        if got != n:
            raise ValueError('bad TFRecord file {} (decoded {} of {})'.format(path, got, n))
        return out
    imgs = []
    for rec in iter_records(path):
        imgs.append(parse_image_record(rec))
        if max_images is not None and len(imgs) >= max_images:
            break
    return np.stack(imgs)


class TFRecordImageDataset:
    """All levels of detail of a TFRecord directory, decoded into host uint8 arrays.

    ``images[lod]`` is ``[N, C, r, r]`` with r = resolution / 2**lod.  Small image-generation
    datasets (MNIST/CIFAR scale) fit in host memory many times over; the model uploads the level
    it trains on to HBM once per level change.
    """

    def __init__(self, tfrecord_dir: str, max_label_size='full', max_images: Optional[int] = None):
        if not os.path.isdir(tfrecord_dir):
            raise FileNotFoundError(tfrecord_dir)
        files = sorted(glob.glob(os.path.join(tfrecord_dir, '*.tfrecords')))
        if not files:
            raise ValueError('no *.tfrecords in {}'.format(tfrecord_dir))
        per_file = {p: _read_images(p, max_images) for p in files}
        shapes = {p: a.shape[1:] for p, a in per_file.items()}
        max_shape = max(shapes.values(), key=lambda s: int(np.prod(s)))
        self.resolution = int(max_shape[1])
        self.resolution_log2 = int(np.log2(self.resolution))
        self.shape = [int(max_shape[0]), self.resolution, self.resolution]
        self.images: Dict[int, np.ndarray] = {}
        for p, a in per_file.items():
            s = shapes[p]
            assert s[0] == max_shape[0] and s[1] == s[2], s
            self.images[self.resolution_log2 - int(np.log2(s[1]))] = a
        for lod in range(self.resolution_log2 - 1):
            if lod not in self.images:
                raise ValueError('missing level of detail {} in {}'.format(lod, tfrecord_dir))
        self.labels = np.zeros((len(self.images[0]), 0), np.float32)
        guess = sorted(glob.glob(os.path.join(tfrecord_dir, '*.labels')))
        if guess and max_label_size != 0:
            lab = np.load(guess[0], allow_pickle=False)
            assert lab.ndim == 2
            if max_label_size != 'full':
                lab = lab[:, :int(max_label_size)]
            self.labels = lab.astype(np.float32)[:len(self.images[0])]
        self.label_size = int(self.labels.shape[1])
        self.dynamic_range = [0, 255]

    @property
    def num_images(self):
        return int(self.images[0].shape[0])

    def level(self, lod: int) -> np.ndarray:
        return self.images[int(lod)]
