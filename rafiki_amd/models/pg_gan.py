"""PgGan — Progressive Growing of GANs (WGAN-GP), the IMAGE_GENERATION example model.

Reference: examples/models/image_generation/pg_gans.py (PG_GANs :34-377, G_paper/D_paper :803-989,
Optimizer :1093-1225, TrainingSchedule :1227-1274, losses :1276-1328).  Same knobs, schedule,
losses, Gs moving average, optimizer-state reset per level of detail, TFRecord dataset format and
predict contract ([grid_w, grid_h, n_images] -> JPEG file paths).  Re-designed for MI355X:

* fp32 by default (the reference's precision, pg_gans.py:830,914): NHWC fp32 activations on the
  v_mfma_f32_32x32x2_f32 kernels (``ops.f32``); ``dtype='bf16'`` (knob or RAFIKI_DTYPE) opts into the
  bf16 MFMA kernels.  Weights live as fp32 masters in a flat arena (``engine.flat``); every conv /
  dense runs through twice-differentiable autograd Functions (``ops.autograd``) — the gradient
  penalty's double backward goes through the same kernels;
* the resampling convs are native: ``Conv0_up`` (upscale2d + conv3x3) is one parity-grouped
  transposed-conv launch reading the half-resolution input, ``Conv1_down`` (conv3x3 + downscale2d)
  one 4x4 stride-2 gather conv — 1/2.25 of the full-resolution MACs, no 2x tensor, and their
  backward passes are the same family; the LOD blends' upscale2d / downscale2d are native kernels;
  the 513-channel minibatch-stddev conv is zero-padded to 520 input channels (MBSTD_PAD = 8; 32 -> 544
  makes its three passes eligible for the pre-split X6 GEMMs too, which measured no faster:
  profiles/pg_gan_mbstd_pad_ab_r6.txt);
* equalized learning rate by re-parameterisation (arena holds c*w, Adam steps with lr*c, eps*c);
* data parallel (``DATA_PARALLEL = True``): when the worker group has N ranks the trial's minibatch
  is split across them (pg_gans.py:290-293) and gradients are averaged by bucketed RCCL
  all-reduces over the flat gradient arena (launched from backward hooks in eager rounds, after the
  captured gradient segment in graphed rounds, untouched buckets skipped)
  (``parallel.grad_bucket``; replaces the per-variable NCCL all-sum at pg_gans.py:1164-1171);
* every rank draws the GLOBAL minibatch's indices / latents / mixing factors from one shared Philox
  stream and keeps its strided shard (the columns of the [group, N/group] minibatch-stddev layout),
  so N ranks x N/N-th of the minibatch compute exactly the 1-rank step (tests/test_pg_gan.py);
* DP rounds on RCCL are captured in hipGraphs like single-GPU rounds, the bucketed all-reduces
  included (``GraphedRounds``);
* mid-trial checkpoint / resume (the reference only pickles at trial end,
  pg_gans.py:219-232): G / D / Gs, both Adam states, the RNG counter and the schedule position,
  saved by rank 0 every ``checkpoint_secs`` and broadcast to every rank on resume;
* the non-finite-gradient guard (pg_gans.py:1180-1191) is a device flag read by the Adam kernel,
  so no host sync per step;
* all work at the native resolution of the current level of detail: the reference upsamples G's
  output to full resolution and D box-filters it back (pg_gans.py:364-369, :1030), an identity
  for integer LOD that we skip.

evaluate(): the reference downloads the Inception-v3 graph to compute an Inception Score; with no
network we compute the same statistic (10-split exp(E KL(p(y|x) || p(y))), pg_gans.py:147-164) with
a classifier trained locally on the evaluation split (its labels if present, otherwise k-means
pseudo-classes).  The number is therefore NOT comparable to a published Inception Score.
"""
from __future__ import annotations

import contextlib
import math
import os
import pickle
import tempfile
import time
import uuid

import numpy as np
import torch

from rafiki_amd.constants import TaskType  # noqa: F401
from rafiki_amd.engine.convnet import default_dtype
from rafiki_amd.engine.flat import FlatAdam, FlatParams, init_const, init_normal
from rafiki_amd.model import BaseModel, CategoricalKnob, FixedKnob, FloatKnob, IntegerKnob, logger
from rafiki_amd.ops import _lib, autograd as A, f32 as S
from rafiki_amd.ops.graphs import capture as _capture, device_sync
from rafiki_amd.parallel.context import current as trial_context


def _pad8(n):
    return (int(n) + 7) // 8 * 8


# input channels of the minibatch-stddev conv (512 + 1) are zero-padded to a multiple of this (the
# Winograd paths need C % 8 == 0; 32 would also admit the pre-split X6 GEMMs, whose K step is 32: same-box
# lod 3 3.90 / 3.91 ms at 32 vs 3.88 / 3.89 at 8, profiles/pg_gan_mbstd_pad_ab_r6.txt)
MBSTD_PAD = int(os.environ.get('RAFIKI_MBSTD_PAD', '8'))
# the Gs EMA over the G ranges that ever trained only (bit-identical; RAFIKI_GS_TRIM=0: the whole arena)
GS_TRIM = os.environ.get('RAFIKI_GS_TRIM', '1') != '0'


# ============================================================================== networks
class PgNetworks:
    """G, D (trainable, flat arenas) and Gs (EMA of G) for one resolution/channel configuration."""

    def __init__(self, num_channels=1, resolution=32, label_size=0, fmap_base=8192, fmap_decay=1.0, fmap_max=512,
                 latent_size=None, mbstd_group_size=4, device='cpu', seed=0, dtype='fp32'):
        self.num_channels, self.resolution, self.label_size = int(num_channels), int(resolution), int(label_size)
        self.L = int(np.log2(resolution))
        assert resolution == 2 ** self.L and resolution >= 4, resolution
        self.fmap_base, self.fmap_decay, self.fmap_max = fmap_base, fmap_decay, fmap_max
        self.latent_size = int(latent_size or self.nf(0))
        self.mbstd_group_size = int(mbstd_group_size)
        self.device = torch.device(device)
        self.dtype = dtype
        bf = dtype == 'bf16'
        # activation dtype of the GPU path (CPU: the fp32 PyTorch reference)
        self.act_dtype = torch.bfloat16 if (bf and self.device.type == 'cuda') else torch.float32
        self.cpad = _pad8(self.num_channels)
        self.combo = self.latent_size + self.label_size
        self.combo_p = _pad8(self.combo)
        self.dout_p = _pad8(1 + self.label_size)
        self.G = FlatParams(self.device, seed, compute_bf16=bf)
        self.D = FlatParams(self.device, seed + 1, compute_bf16=bf)
        self._define_G()
        self._define_D()
        self.G.build()
        self.D.build()
        self.Gs_master = self.G.master.clone()
        self.Gs_bf16 = self.Gs_master.to(torch.bfloat16) if bf else None
        # G parameters whose Gs may differ from G (None: any): Gs starts as a bit copy of G, and a weight
        # Adam never touched keeps Gs == G exactly under the EMA, so update_Gs may skip it
        self.gs_moved = set()
        self.g_params = self._leaves(self.G)
        self.d_params = self._leaves(self.D)

    def nf(self, stage):
        return min(int(self.fmap_base / (2.0 ** (stage * self.fmap_decay))), self.fmap_max)

    # -- parameter definition (equalized LR: effective weight ~ N(0, std^2), lr multiplier = std)
    @staticmethod
    def _w(flat, name, shape, fan_in, gain=math.sqrt(2.0), zero_cols=None, zero_rows=None, bias_shape=None):
        std = gain / math.sqrt(fan_in)

        def init(t, g):
            t.normal_(0.0, std, generator=g)
            if zero_rows is not None:
                t[zero_rows] = 0.0
            if zero_cols is not None:
                t[..., zero_cols] = 0.0
        flat.add(name + '/weight', shape, init, decay=True, lr_mult=std)
        flat.add(name + '/bias', bias_shape or (shape[0],), init_const(0.0), decay=False)

    def _define_G(self):
        G, nc = self.G, self.num_channels
        n1 = self.nf(1)
        # 4x4 dense: [16*nf(1), combo_p] (rows laid out (h, w, c) = NHWC), bias per channel
        self._w(G, '4x4/Dense', (16 * n1, self.combo_p), self.combo, gain=math.sqrt(2) / 4,
                zero_cols=slice(self.combo, None) if self.combo_p > self.combo else None,
                bias_shape=(n1,))  # per-channel bias, applied after the NHWC reshape
        self._w(G, '4x4/Conv', (n1, 9 * n1), 9 * n1)
        for res in range(3, self.L + 1):
            cin, cout = self.nf(res - 2), self.nf(res - 1)
            self._w(G, '%dx%d/Conv0_up' % (2 ** res, 2 ** res), (cout, 9 * cin), 9 * cin)
            self._w(G, '%dx%d/Conv1' % (2 ** res, 2 ** res), (cout, 9 * cout), 9 * cout)
        for res in range(2, self.L + 1):
            c = self.nf(res - 1)
            self._w(G, 'ToRGB_lod%d' % (self.L - res), (self.cpad, c), c, gain=1.0,
                    zero_rows=slice(nc, None) if self.cpad > nc else None)

    def _define_D(self):
        D, nc = self.D, self.num_channels
        for res in range(2, self.L + 1):
            c = self.nf(res - 1)
            self._w(D, 'FromRGB_lod%d' % (self.L - res), (c, self.cpad), nc,
                    zero_cols=slice(nc, None) if self.cpad > nc else None)
        for res in range(self.L, 2, -1):
            c0, c1 = self.nf(res - 1), self.nf(res - 2)
            self._w(D, '%dx%d/Conv0' % (2 ** res, 2 ** res), (c0, 9 * c0), 9 * c0)
            self._w(D, '%dx%d/Conv1_down' % (2 ** res, 2 ** res), (c1, 9 * c0), 9 * c0)
        n1, n0 = self.nf(1), self.nf(0)
        cm = n1 + 1 if self.mbstd_group_size > 1 else n1
        cm_p = (cm + MBSTD_PAD - 1) // MBSTD_PAD * MBSTD_PAD
        self.mbstd_cp = cm_p
        # [Cout][tap][Cin_p] with the padded input channels zeroed
        D.add('4x4/Conv/weight', (n1, 9, cm_p), _zero_tail_init(math.sqrt(2) / math.sqrt(9 * cm), cm),
              decay=True, lr_mult=math.sqrt(2) / math.sqrt(9 * cm))
        D.add('4x4/Conv/bias', (n1,), init_const(0.0), decay=False)
        self._w(D, '4x4/Dense0', (n0, 16 * n1), 16 * n1)
        self._w(D, '4x4/Dense1', (self.dout_p, n0), n0, gain=1.0,
                zero_rows=slice(1 + self.label_size, None) if self.dout_p > 1 + self.label_size else None)

    @staticmethod
    def _leaves(flat):
        out = {}
        for s in flat.specs:
            p = torch.nn.Parameter(flat.w(s.name))
            p.grad = flat.g(s.name)
            out[s.name] = p
        return out

    # -- parameter sources
    def src_G(self):
        return _Src(self.g_params, lambda n: self.G.wb(n) if self.Gs_bf16 is not None else None)

    def src_Gs(self):
        return _Src({s.name: _view(self.Gs_master, s) for s in self.G.specs},
                    lambda n: _view(self.Gs_bf16, self.G._by_name[n]) if self.Gs_bf16 is not None else None)

    def src_D(self):
        return _Src(self.d_params, lambda n: self.D.wb(n) if self.Gs_bf16 is not None else None)

    def set_requires_grad(self, params, flag):
        for p in params.values():
            p.requires_grad_(flag)

    # -- forward passes ------------------------------------------------------------------
    def _conv(self, P, name, x, taps=9, lrelu=None):
        w = P.w(name + '/weight')
        return A.conv2d(x, w.reshape(w.shape[0], -1), P.w(name + '/bias'), taps=taps,
                        wb=_maybe2d(P.wb(name + '/weight'), w), lrelu=lrelu)

    def _upconv(self, P, name, x):
        w = P.w(name + '/weight')
        return A.upscale_conv2d(x, w, P.w(name + '/bias'), wb=_maybe2d(P.wb(name + '/weight'), w))

    def _conv_down(self, P, name, x, lrelu=None):
        w = P.w(name + '/weight')
        return A.conv2d_downscale2d(x, w.reshape(w.shape[0], -1), P.w(name + '/bias'),
                                    wb=_maybe2d(P.wb(name + '/weight'), w), lrelu=lrelu)

    def _dense(self, P, name, x, bias=True, lrelu=None):
        w = P.w(name + '/weight')
        return A.dense(x, w, P.w(name + '/bias') if bias else None, wb=P.wb(name + '/weight'), lrelu=lrelu)

    def live_names(self, lod):
        """(G names, D names): the parameters the generator / discriminator use at ``lod`` (the layers
        ``generator`` / ``discriminator`` below evaluate); the others get no gradient that round."""
        cur = self.L - int(math.floor(lod))
        frac = lod - math.floor(lod)
        g = ['4x4/Dense', '4x4/Conv', 'ToRGB_lod%d' % (self.L - cur)]
        d = ['FromRGB_lod%d' % (self.L - cur), '4x4/Conv', '4x4/Dense0', '4x4/Dense1']
        for res in range(3, cur + 1):
            tag = '%dx%d' % (2 ** res, 2 ** res)
            g += [tag + '/Conv0_up', tag + '/Conv1']
            d += [tag + '/Conv0', tag + '/Conv1_down']
        if frac > 0 and cur > 2:
            g.append('ToRGB_lod%d' % (self.L - cur + 1))
            d.append('FromRGB_lod%d' % (self.L - cur + 1))
        return ([n + s for n in g for s in ('/weight', '/bias')], [n + s for n in d for s in ('/weight', '/bias')])

    def generator(self, P, latents, labels, lod):
        """latents [N, latent] fp32, labels [N, label_size] -> images NHWC [N, r, r, cpad] (bf16 on GPU)
        at r = 2 ** (L - floor(lod)), in [-1, 1] drange (pg_gans.py:803-880, 'recursive' structure)."""
        dt = self.act_dtype
        PN, LPN = A.pixel_norm, A.lrelu_pixel_norm
        N = latents.shape[0]
        combo = torch.cat([latents, labels], 1) if self.label_size else latents
        combo = combo.float()
        if combo.is_cuda and combo.shape[-1] % 8 == 0 and combo.shape[-1] <= 1024:
            combo = LPN(combo, None, slope=1.0)   # pixel norm: the fused kernel with the identity activation
        else:
            combo = PN(combo)
        if self.combo_p > self.combo:
            combo = torch.cat([combo, combo.new_zeros(N, self.combo_p - self.combo)], 1)
        x = self._dense(P, '4x4/Dense', combo.to(dt), bias=False).reshape(N, 4, 4, self.nf(1))
        x = LPN(x, P.w('4x4/Dense/bias'))
        x = LPN(self._conv(P, '4x4/Conv', x))
        cur = self.L - int(math.floor(lod))
        frac = lod - math.floor(lod)
        prev = None
        for res in range(3, cur + 1):
            prev = x
            tag = '%dx%d' % (2 ** res, 2 ** res)
            x = LPN(self._upconv(P, tag + '/Conv0_up', x))
            x = LPN(self._conv(P, tag + '/Conv1', x))
        img = self._conv(P, 'ToRGB_lod%d' % (self.L - cur), x, taps=1)
        if frac > 0 and cur > 2:
            lo = A.upscale2d(self._conv(P, 'ToRGB_lod%d' % (self.L - cur + 1), prev, taps=1))
            img = img + (lo - img) * frac
        return img

    def discriminator(self, P, img, lod, segs=1, raw=False):
        """img NHWC [N, r, r, cpad] at the current LOD resolution -> (scores [N] fp32, label logits).
        ``segs`` > 1: img stacks that many independent minibatches (one batched evaluation;
        minibatch-stddev groups stay inside each).  ``raw``: the fp32 output rows [N, dout_p] instead
        (score in column 0, label logits after it) — the fused loss head reads them in place."""
        cur = self.L - int(math.floor(lod))
        frac = lod - math.floor(lod)
        x = self._conv(P, 'FromRGB_lod%d' % (self.L - cur), img, taps=1, lrelu=0.2)
        for res in range(cur, 2, -1):
            tag = '%dx%d' % (2 ** res, 2 ** res)
            x = self._conv(P, tag + '/Conv0', x, lrelu=0.2)
            x = self._conv_down(P, tag + '/Conv1_down', x, lrelu=0.2)
            if res == cur and frac > 0:
                y = self._conv(P, 'FromRGB_lod%d' % (self.L - res + 1), A.downscale2d(img), taps=1, lrelu=0.2)
                x = x + (y - x) * frac
        if self.mbstd_group_size > 1:
            x = A.minibatch_stddev(x, self.mbstd_group_size, pad_to=MBSTD_PAD, segs=segs)
        x = self._conv(P, '4x4/Conv', x, lrelu=0.2)
        N = x.shape[0]
        x = self._dense(P, '4x4/Dense0', x.reshape(N, -1), lrelu=0.2)
        out = self._dense(P, '4x4/Dense1', x).float()
        if raw:
            return out
        return out[:, 0], out[:, 1:1 + self.label_size]

    # -- Gs moving average (pg_gans.py:1247 setup_as_moving_average_of, beta = G_smoothing)
    def update_Gs(self, beta, table=None):
        """Gs <- G + (Gs - G) * beta; ``table`` (a SegTable over the G ranges that ever trained, see
        PgGan._gs_table): the same update over those ranges only — bit-identical, since everywhere else
        G - Gs is exactly zero."""
        if self.device.type == 'cuda':
            from rafiki_amd.ops import functional as F
            if table is not None:
                F.lerp_multi(self.Gs_master, self.G.master, beta, table, dst_bf16=self.Gs_bf16)
                return
            F.lerp_(self.Gs_master, self.G.master, beta, dst_bf16=self.Gs_bf16)
        else:
            self.Gs_master.copy_(self.G.master + (self.Gs_master - self.G.master) * beta)
            if self.Gs_bf16 is not None:
                self.Gs_bf16.copy_(self.Gs_master)

    def state(self):
        return {'G': self.G.state_dict(),
                'D': self.D.state_dict(),
                'Gs': {s.name: _view(self.Gs_master, s).detach().cpu().numpy().copy() for s in self.G.specs}}

    def load_state(self, st):
        self.gs_moved = None   # a restored Gs may differ from G anywhere
        self.G.load_state_dict(st['G'])
        self.D.load_state_dict(st['D'])
        for s in self.G.specs:
            if s.name in st['Gs']:
                _view(self.Gs_master, s).copy_(torch.as_tensor(st['Gs'][s.name]).reshape(s.shape))
        if self.Gs_bf16 is not None:
            self.Gs_bf16.copy_(self.Gs_master)


def _zero_tail_init(std, real_c):
    def f(t, g):
        t.normal_(0.0, std, generator=g)
        t[..., real_c:] = 0.0
    return f


def _view(buf, spec):
    return buf[spec.offset:spec.offset + spec.numel].view(spec.shape)


def _maybe2d(wb, w):
    return None if wb is None else wb.reshape(w.shape[0], -1)


class _Src:
    def __init__(self, params, wb_fn):
        self.params, self.wb_fn = params, wb_fn

    def w(self, name):
        return self.params[name]

    def wb(self, name):
        return self.wb_fn(name) if self.params[name].device.type == 'cuda' else None


# ============================================================================== schedule
class TrainingSchedule:
    """pg_gans.py:1227-1274 (minibatch dicts per minibatch_base, LOD phases, per-GPU caps)."""

    MINIBATCH_DICTS = {
        4: {4: 128, 8: 128, 16: 128, 32: 64, 64: 32, 128: 16, 256: 8, 512: 4},
        8: {4: 256, 8: 256, 16: 128, 32: 64, 64: 32, 128: 16, 256: 8},
        16: {4: 512, 8: 256, 16: 128, 32: 64, 64: 32, 128: 16},
        32: {4: 512, 8: 256, 16: 128, 32: 64, 64: 32},
    }

    def __init__(self, cur_nimg, resolution_log2, num_gpus=1, lod_initial_resolution=4, lod_training_kimg=600,
                 lod_transition_kimg=600, minibatch_base=16, max_minibatch_per_gpu=None, G_lrate=0.001,
                 D_lrate=0.001):
        if max_minibatch_per_gpu is None:
            max_minibatch_per_gpu = {256: 16, 512: 8, 1024: 4}
        mb_dict = self.MINIBATCH_DICTS.get(int(minibatch_base), {})
        self.kimg = cur_nimg / 1000.0
        phase_dur = lod_training_kimg + lod_transition_kimg
        phase_idx = int(np.floor(self.kimg / phase_dur)) if phase_dur > 0 else 0
        phase_kimg = self.kimg - phase_idx * phase_dur
        lod = float(resolution_log2)
        lod -= np.floor(np.log2(lod_initial_resolution))
        lod -= phase_idx
        if lod_transition_kimg > 0:
            lod -= max(phase_kimg - lod_training_kimg, 0.0) / lod_transition_kimg
        self.lod = max(float(lod), 0.0)
        self.resolution = 2 ** (resolution_log2 - int(np.floor(self.lod)))
        mb = mb_dict.get(self.resolution, int(minibatch_base))
        mb -= mb % num_gpus
        if self.resolution in max_minibatch_per_gpu:
            mb = min(mb, max_minibatch_per_gpu[self.resolution] * num_gpus)
        self.minibatch = int(mb)
        self.G_lrate, self.D_lrate = float(G_lrate), float(D_lrate)


# ============================================================================== dataset
def load_gan_dataset(dataset_uri):
    """TFRecord directory (reference format), IMAGE_FILES zip, or synthetic:// URI ->
    TFRecordImageDataset-like object with .images[lod] uint8 [N, C, r, r] and .labels."""
    from rafiki_amd.model import tfrecord as T
    from rafiki_amd.model import dataset_utils
    uri = str(dataset_uri)
    path = uri[7:] if uri.startswith('file://') else uri
    if os.path.isdir(os.path.expanduser(path)):
        return T.TFRecordImageDataset(os.path.expanduser(path))
    ds = dataset_utils.load_dataset_of_image_files(uri)
    imgs, labels = ds.as_arrays()
    imgs = np.asarray(imgs)
    if imgs.ndim == 3:
        imgs = imgs[:, None]
    else:
        imgs = imgs.transpose(0, 3, 1, 2)
    return _ArrayPyramid(imgs, labels)


class _ArrayPyramid:
    def __init__(self, imgs, labels=None):
        from rafiki_amd.model.tfrecord import downscale_images
        R = imgs.shape[-1]
        self.resolution = R
        self.resolution_log2 = int(np.log2(R))
        assert R == 2 ** self.resolution_log2 and imgs.shape[-2] == R, imgs.shape
        self.shape = [imgs.shape[1], R, R]
        self.images = {0: imgs.astype(np.uint8)}
        cur = imgs.astype(np.float32)
        for lod in range(1, self.resolution_log2 - 1):
            cur = downscale_images(cur)
            self.images[lod] = np.rint(cur).clip(0, 255).astype(np.uint8)
        if labels is not None and len(labels):
            labels = np.asarray(labels).astype(np.int64)
            oh = np.zeros((len(labels), int(labels.max()) + 1), np.float32)
            oh[np.arange(len(labels)), labels] = 1.0
            self.class_labels = labels
        else:
            oh = np.zeros((len(imgs), 0), np.float32)
            self.class_labels = None
        self.labels = oh
        self.label_size = 0  # IMAGE_FILES labels are used for evaluation only (unconditional GAN)
        self.dynamic_range = [0, 255]

    @property
    def num_images(self):
        return int(self.images[0].shape[0])


# ============================================================================== model
class TrialRng:
    """Per-trial random source.  GPU: the Philox HIP kernel keyed by (seed, call-site stream id,
    device step counter) — a captured training round bumps the counter itself, so graph replays
    draw fresh latents / indices / mixing factors with no host work.  CPU: a torch.Generator."""

    # call-site stream ids
    D_IDX, D_LAT, D_ALPHA, G_LAB, G_LAT = 1, 2, 3, 4, 5

    def __init__(self, device, seed):
        self.device, self.seed = device, int(seed)
        if device.type == 'cuda':
            self.step = torch.zeros(1, dtype=torch.int32, device=device)
        else:
            self.gen = torch.Generator()
            self.gen.manual_seed(self.seed)

    def _draw(self, shape, dist, sid, hi=0):
        from rafiki_amd.ops import functional as F
        out = torch.empty(shape, dtype=torch.int32 if dist == F.RNG_RANDINT else torch.float32, device=self.device)
        return F.philox_(out, dist, seed=self.seed, stream_id=sid, step=self.step, hi=hi)

    def randint(self, hi, n, sid):
        if self.device.type == 'cuda':
            from rafiki_amd.ops import functional as F
            return self._draw((n,), F.RNG_RANDINT, sid, hi=hi)
        return torch.randint(0, hi, (n,), generator=self.gen)

    def randn(self, shape, sid):
        if self.device.type == 'cuda':
            from rafiki_amd.ops import functional as F
            return self._draw(shape, F.RNG_NORMAL, sid)
        return torch.randn(shape, generator=self.gen)

    def rand(self, shape, sid):
        if self.device.type == 'cuda':
            from rafiki_amd.ops import functional as F
            return self._draw(shape, F.RNG_UNIFORM, sid)
        return torch.rand(shape, generator=self.gen)

    def advance(self):
        if self.device.type == 'cuda':
            from rafiki_amd.ops import functional as F
            F.add_int_(self.step, 1)


def grad_bucket_mb() -> float:
    """PG-GAN's data-parallel bucket size: 4 MiB (RAFIKI_GRAD_BUCKET_MB overrides) — each 3x3x512x512 conv
    is a bucket of its own, so the lod-3 rounds skip every untouched block exactly and start reducing early
    (docs/architecture.md, comm model; profiles/pggan_comm_model_r6.json)."""
    return float(os.environ.get('RAFIKI_GRAD_BUCKET_MB', 4))


class GraphedRounds:
    """hipGraph cache of training rounds (D_repeats D steps + Gs EMA + one G step).

    A round's shapes, learning rates and LOD are static inside a stable LOD phase, so the first
    round with a new key runs eagerly (it also autotunes every GEMM shape), the second one is
    captured, and every later round is one graph replay — the PG-GAN step at 4x4 is otherwise
    bound by host-side launch overhead of ~600 small kernels.  Randomness comes from TrialRng's
    device counter, the Adam step count lives on the device, and the loss accumulators are
    persistent buffers, so replays need no host input."""

    def __init__(self, enabled, collectives=False):
        self.enabled = enabled
        self.collectives = collectives
        self.graphs = {}
        self.seen = set()
        self.captures = 0

    def clear(self):
        from ..ops.graphs import quiesced
        with quiesced():
            self.graphs.clear()
        self.seen.clear()

    def run_segments(self, key, segs):
        """A round as a list of ('g', fn) compute segments, ('s', BucketedGrads) gradient segments and
        ('e', fn) eager collective segments (data-parallel rounds: gradients -> all-reduce -> optimizer).
        Each compute segment becomes its own graph; a gradient segment becomes a SEQUENCE of graphs
        cut where a gradient bucket completes, and its bucket all-reduces are launched eagerly between
        their replays, so they run on RCCL's stream while the rest of the backward replays (one memory
        pool per key, everything replayed in capture order).  No collective is ever inside a capture
        and the process group's watchdog has nothing of ours to race (no sleep, deterministic)."""
        if not self.enabled:
            for _, fn in segs:
                fn()
            return
        gs = self.graphs.get(key)
        if gs is not None:
            for (kind, fn), g in zip(segs, gs):
                if kind == 's':
                    fn.replay(g)
                elif g is None:
                    fn()
                else:
                    g.replay()
            return
        if key not in self.seen or any(kind == 's' and not fn.planned for kind, fn in segs):
            # eager until every gradient segment's bucket plan is traced (BucketedGrads.TRACES runs)
            self.seen.add(key)
            for _, fn in segs:
                fn()
            return
        device_sync()
        pool = torch.cuda.graph_pool_handle()
        gs = []
        for kind, fn in segs:
            if kind == 'e':
                fn()
                gs.append(None)
                continue
            if kind == 's':
                parts = fn.capture(pool)
                fn.replay(parts)   # a capture records, it does not execute: run it (and its reduces) now
                gs.append(parts)
                self.captures += len(parts)
                continue
            g = torch.cuda.CUDAGraph()
            with _capture(g, pool=pool):
                fn()
            g.replay()   # a capture records, it does not execute: run it before the next segment
            gs.append(g)
            self.captures += 1
        self.graphs[key] = gs

    def run(self, key, fn):
        if not self.enabled:
            fn()
            return
        g = self.graphs.get(key)
        if g is not None:
            g.replay()
            return
        if key not in self.seen:
            self.seen.add(key)
            fn()
            return
        g = torch.cuda.CUDAGraph()
        device_sync()
        if self.collectives:
            # opt-in path (see the RAFIKI_PGGAN_GRAPH_COLLECTIVES note in PgGan.train): give the process
            # group's watchdog ~3 poll periods to retire the eager rounds' completed works before the
            # capture starts.  Residual race: a stalled watchdog thread could still poll during it.
            time.sleep(0.3)
        with _capture(g):
            fn()
        self.graphs[key] = g
        self.captures += 1
        g.replay()


class PgGan(BaseModel):
    DATA_PARALLEL = True

    @staticmethod
    def get_knob_config():
        return {
            'D_repeats': IntegerKnob(1, 3),
            'minibatch_base': CategoricalKnob([4, 8, 16, 32]),
            'G_lrate': FloatKnob(1e-3, 3e-3, is_exp=False),
            'D_lrate': FloatKnob(1e-3, 3e-3, is_exp=False),
            'lod_initial_resolution': FixedKnob(4),
            'total_kimg': FixedKnob(2),
            'lod_training_kimg': FixedKnob(600),
            'lod_transition_kimg': FixedKnob(600),
        }

    def __init__(self, **knobs):
        super().__init__(**knobs)
        self._knobs = dict(knobs)
        ctx = trial_context()
        self.ctx = ctx
        self.device = ctx.device
        self.world = ctx.world_size
        self.rank = ctx.rank
        self.nets = None
        self.lod = None
        self._meta = {}
        self.seed = int(knobs.get('seed', 1000))
        self.stats = {}

    # ------------------------------------------------------------------ helpers
    def _k(self, name, default):
        return self._knobs.get(name, default)

    def _build(self, shape, label_size):
        self._meta = dict(num_channels=int(shape[0]), resolution=int(shape[1]), label_size=int(label_size),
                          fmap_base=int(self._k('fmap_base', 8192)), fmap_max=int(self._k('fmap_max', 512)),
                          mbstd_group_size=int(self._k('mbstd_group_size', 4)),
                          dtype=str(self._k('dtype', default_dtype())))
        self.nets = PgNetworks(device=self.device, seed=self.seed, **self._meta)
        if self.world > 1:
            import torch.distributed as dist
            for buf in (self.nets.G.master, self.nets.D.master):
                dist.broadcast(buf, src=0)
            self.nets.G.sync_bf16()
            self.nets.D.sync_bf16()
            self.nets.Gs_master.copy_(self.nets.G.master)
            if self.nets.Gs_bf16 is not None:
                self.nets.Gs_bf16.copy_(self.nets.Gs_master)

    def _reals(self, level_u8, idx, frac):
        """uint8 [N, C, r, r] (device) rows idx -> NHWC [n, r, r, cpad] in [-1, 1] with LOD fade
        (pg_gans.py:347-369 process_reals: dynamic range, FadeLOD; UpscaleLOD is the identity here)."""
        nets = self.nets
        if (self.device.type == 'cuda' and frac <= 0 and nets.act_dtype == torch.float32 and level_u8.is_cuda
                and idx.dtype == torch.int32):
            # the minibatch gather folded into the pack kernel (no index_select pass)
            return S.pack_nhwc(level_u8, nets.cpad, 2.0 / 255.0, -1.0, idx=idx)
        x = level_u8.index_select(0, idx)
        if self.device.type == 'cuda' and frac <= 0:
            from rafiki_amd.ops import functional as F
            pack = S.pack_nhwc if nets.act_dtype == torch.float32 else F.pack_nhwc
            return pack(x.contiguous(), nets.cpad, 2.0 / 255.0, -1.0)
        x = x.float() * (2.0 / 255.0) - 1.0
        if frac > 0:
            N, C, r, _ = x.shape
            y = x.reshape(N, C, r // 2, 2, r // 2, 2).mean((3, 5), keepdim=True).expand(N, C, r // 2, 2, r // 2, 2)
            x = x + (y.reshape(N, C, r, r) - x) * frac
        x = x.permute(0, 2, 3, 1)
        if nets.cpad > x.shape[-1]:
            x = torch.cat([x, x.new_zeros(*x.shape[:3], nets.cpad - x.shape[-1])], -1)
        return x.to(nets.act_dtype).contiguous()

    def _slice_images(self, img):
        return img[..., :self.nets.num_channels]

    # ------------------------------------------------------------------ train
    def _shard(self, t):
        """Rank's part of a global-minibatch draw: the global batch is laid out [g, world, mb/g] in
        minibatch-stddev group order (sample n -> group n % (N/g)), and a rank keeps its column block,
        so every mbstd group lives on one rank and the local grouping reproduces the global one."""
        if self.world == 1:
            return t
        mb = t.shape[0] // self.world
        g = min(self.nets.mbstd_group_size, mb)
        return t.reshape(g, self.world, mb // g, *t.shape[1:])[:, self.rank].reshape(mb, *t.shape[1:])

    # ------------------------------------------------------------------ checkpoint / resume
    def _ckpt_state(self, G_opt, D_opt, rng, cur_nimg, prev_lod, tick):
        nets = self.nets

        def host(t):
            return t.detach().cpu().numpy().copy()
        st = {'G': host(nets.G.master), 'D': host(nets.D.master), 'Gs': host(nets.Gs_master),
              'opt': {k: [host(o.m), host(o.v), host(o.t)] for k, o in (('G', G_opt), ('D', D_opt))},
              'cur_nimg': int(cur_nimg), 'prev_lod': float(prev_lod), 'tick': int(tick), 'stats': dict(self.stats),
              'meta': dict(self._meta)}
        st['rng'] = host(rng.step) if rng.device.type == 'cuda' else rng.gen.get_state().numpy().copy()
        return st

    def _restore_ckpt(self, st, G_opt, D_opt, rng):
        nets = self.nets
        nets.G.master.copy_(torch.as_tensor(st['G']))
        nets.D.master.copy_(torch.as_tensor(st['D']))
        nets.Gs_master.copy_(torch.as_tensor(st['Gs']))
        nets.G.sync_bf16()
        nets.D.sync_bf16()
        if nets.Gs_bf16 is not None:
            nets.Gs_bf16.copy_(nets.Gs_master)
        for k, o in (('G', G_opt), ('D', D_opt)):
            for t, v in zip((o.m, o.v, o.t), st['opt'][k]):
                t.copy_(torch.as_tensor(v))
        if rng.device.type == 'cuda':
            rng.step.copy_(torch.as_tensor(st['rng']))
        else:
            rng.gen.set_state(torch.as_tensor(st['rng']))
        self.stats = dict(st['stats'])
        return int(st['cur_nimg']), float(st['prev_lod']), int(st['tick'])

    def train(self, dataset_uri, **overrides):
        from rafiki_amd.parallel import dist as D
        from rafiki_amd.parallel.grad_bucket import FlatGradAllReduce
        from rafiki_amd.utils import faults
        knobs = dict(self._knobs, **overrides)
        ds = load_gan_dataset(dataset_uri)
        if self.nets is None:
            self._build(ds.shape, ds.label_size)
        nets, dev = self.nets, self.device
        total_kimg = float(knobs.get('total_kimg', 2))
        D_repeats = int(knobs.get('D_repeats', 1))
        minibatch_repeats = int(knobs.get('minibatch_repeats', 4))
        G_smoothing = float(knobs.get('G_smoothing', 0.99))
        sched_kw = dict(lod_initial_resolution=int(knobs.get('lod_initial_resolution', 4)),
                        lod_training_kimg=float(knobs.get('lod_training_kimg', 600)),
                        lod_transition_kimg=float(knobs.get('lod_transition_kimg', 600)),
                        minibatch_base=int(knobs.get('minibatch_base', 16)),
                        G_lrate=float(knobs.get('G_lrate', 1e-3)), D_lrate=float(knobs.get('D_lrate', 1e-3)))
        G_opt = FlatAdam(nets.G, sched_kw['G_lrate'], betas=(0.0, 0.99), eps=1e-8)
        D_opt = FlatAdam(nets.D, sched_kw['D_lrate'], betas=(0.0, 0.99), eps=1e-8)
        for opt in (G_opt, D_opt):
            opt.skip_flag = torch.zeros(1, dtype=torch.int32, device=dev)
        g_ar = d_ar = None
        # force_grad_allreduce: run the bucketed all-reduce path even on one rank (a 1-rank RCCL
        # group rehearses capture of the DP round on a single GPU)
        if self.world > 1 or bool(knobs.get('force_grad_allreduce', False)):
            force = self.world == 1
            # 4 MiB buckets: at lod 3 only a third of the arena receives gradients, and the finer buckets
            # both skip more of the untouched blocks and start reducing earlier in the backward
            # (docs/architecture.md, comm model); RAFIKI_GRAD_BUCKET_MB / the knob override it
            bmb = knobs.get('grad_bucket_mb', grad_bucket_mb())
            g_ar = FlatGradAllReduce(nets.G.grad, nets.G.param_ranges(), list(nets.g_params.values()), self.world,
                                     force=force, bucket_mb=float(bmb))
            d_ar = FlatGradAllReduce(nets.D.grad, nets.D.param_ranges(), list(nets.d_params.values()), self.world,
                                     force=force, bucket_mb=float(bmb))
        rng = TrialRng(dev, self.seed * 7919)   # one stream for all ranks; each keeps its shard
        # RCCL collectives are graph-capturable, gloo ones are not (a gloo group on GPUs is the
        # one-box multi-rank rehearsal: eager)
        # Data-parallel rounds are captured by SEGMENTS (round_segments): each gradient pass as a sequence
        # of graphs cut where a gradient bucket completes, its bucket all-reduces launched eagerly between
        # those replays (overlapping the rest of the backward), then the optimizer graph — no collective
        # is ever inside a capture, so the process group's watchdog has nothing of ours to race, and a
        # gloo group (the one-box multi-rank rehearsal) is capturable too.  The older whole-round capture
        # with the collectives inside stays an opt-in (RAFIKI_PGGAN_GRAPH_COLLECTIVES=1, nccl only): the
        # watchdog polls the eager rounds' completed works on its own schedule, so that capture waits
        # 0.3 s (~3 watchdog periods) first — a residual race, not a guarantee.
        whole = g_ar is not None and (self.ctx.dist.backend == 'nccl'
                                      and os.environ.get('RAFIKI_PGGAN_GRAPH_COLLECTIVES', '0') == '1')
        # dp_segmented=False (tests): the unsegmented round — hooks launch the buckets, finish() waits
        segmented = g_ar is not None and not whole and bool(knobs.get('dp_segmented', True))
        capturable = g_ar is None or whole or segmented
        graphs = GraphedRounds(dev.type == 'cuda' and capturable and bool(knobs.get('cuda_graph', True))
                               and os.environ.get('RAFIKI_PGGAN_GRAPH', '1') != '0', collectives=whole)
        self.segmented = segmented
        self.graphs = graphs
        acc = torch.zeros(6, dtype=torch.float32, device=dev)
        level_cache = {}
        labels_all = torch.as_tensor(ds.labels, device=dev)
        cur_nimg, prev_lod, tick = 0, -1.0, 0
        ck = self.ctx.checkpoint if self.rank == 0 else None
        saved = ck.load() if ck is not None else None
        if self.world > 1:
            saved = D.broadcast_object(self.ctx.dist, saved)
        if saved is not None:
            cur_nimg, prev_lod, tick = self._restore_ckpt(saved['state'], G_opt, D_opt, rng)
            logger.log('resumed from checkpoint at tick {} ({:.3f} kimg)'.format(tick, cur_nimg / 1000.0))
        ckpt_secs = float(knobs.get('checkpoint_secs', 60.0))
        last_ckpt = time.monotonic()
        logger.define_plot('Losses', ['D_loss', 'G_loss'], x_axis='kimg')
        logger.define_plot('Scores', ['real_score', 'fake_score', 'grad_norm'], x_axis='kimg')
        while cur_nimg < total_kimg * 1000:
            sched = TrainingSchedule(cur_nimg, ds.resolution_log2, num_gpus=self.world, **sched_kw)
            lod_int = int(math.floor(sched.lod))
            if lod_int not in level_cache:
                level_cache.clear()
                graphs.clear()
                for ar in (g_ar, d_ar):
                    if ar is not None:
                        ar.clear_plans()
                level_cache[lod_int] = torch.as_tensor(ds.images[lod_int]).to(dev)
            level = level_cache[lod_int]
            if np.floor(sched.lod) != np.floor(prev_lod) or np.ceil(sched.lod) != np.ceil(prev_lod):
                G_opt.reset_state()
                D_opt.reset_state()
                _zero(nets.G.grad)   # ranges that leave the live set keep zero gradients
                _zero(nets.D.grad)
            self.set_lod_live(sched.lod)
            prev_lod = sched.lod
            G_opt.lr, D_opt.lr = sched.G_lrate, sched.D_lrate
            mb = sched.minibatch // self.world
            if mb % min(nets.mbstd_group_size, mb) != 0:
                mb -= mb % nets.mbstd_group_size
            acc.zero_()
            nD = nG = 0
            frac = sched.lod - math.floor(sched.lod)
            key = (sched.lod, mb, G_opt.lr, D_opt.lr, D_repeats, G_smoothing)

            def round_fn():
                self.train_round(sched.lod, mb, level, labels_all, rng, G_opt, D_opt, acc, D_repeats=D_repeats,
                                 G_smoothing=G_smoothing, d_ar=d_ar, g_ar=g_ar)
            segs = (self.round_segments(sched.lod, mb, level, labels_all, rng, G_opt, D_opt, acc,
                                        D_repeats=D_repeats, G_smoothing=G_smoothing, d_ar=d_ar, g_ar=g_ar,
                                        tag=key)
                    if segmented else None)
            for _ in range(minibatch_repeats):
                if frac == 0 and segs is not None:
                    graphs.run_segments(key, segs)
                elif frac == 0:
                    graphs.run(key, round_fn)
                elif segs is not None:   # LOD transition: the fade factor changes every tick, run eagerly
                    for _, fn in segs:
                        fn()
                else:
                    round_fn()
                cur_nimg += sched.minibatch * D_repeats
                nD += D_repeats
                nG += 1
            tick += 1
            a = acc.cpu().numpy()
            self.lod = sched.lod
            self.stats = dict(kimg=cur_nimg / 1000.0, lod=sched.lod, minibatch=sched.minibatch,
                              D_loss=float(a[0] / nD), real_score=float(a[1] / nD), fake_score=float(a[2] / nD),
                              grad_norm=float(a[3] / nD), G_loss=float(a[4] / nG))
            logger.log('tick {}'.format(tick), **self.stats)
            if ck is not None and cur_nimg < total_kimg * 1000 and time.monotonic() - last_ckpt >= ckpt_secs:
                ck.save(self._ckpt_state(G_opt, D_opt, rng, cur_nimg, prev_lod, tick), tick)
                last_ckpt = time.monotonic()
            faults.maybe_fail('crash', tick=tick, rank=self.rank)
        self.lod = prev_lod if prev_lod >= 0 else 0.0
        if g_ar is not None:
            g_ar.remove()
            d_ar.remove()

    def _latents(self, n, rng, sid):
        return self._shard(rng.randn((n * self.world, self.nets.latent_size), sid))

    def _rand_labels(self, labels_all, n, rng):
        if self.nets.label_size == 0:
            return torch.zeros((n, 0), device=self.device)
        idx = self._shard(rng.randint(labels_all.shape[0], n * self.world, TrialRng.G_LAB))
        return labels_all.index_select(0, idx.to(labels_all.device))

    def train_round(self, lod, mb, level, labels_all, rng, G_opt, D_opt, acc, *, D_repeats=1, G_smoothing=0.99,
                    d_ar=None, g_ar=None):
        """D_repeats D steps (each followed by the Gs EMA) then one G step (pg_gans.py:338-342);
        losses accumulate on the device into acc[:4] (D) and acc[4] (G).  Host-sync free, so a
        round is captured whole by GraphedRounds."""
        for _ in range(D_repeats):
            self._d_step(lod, mb, level, labels_all, rng, D_opt, d_ar, acc=acc)
            self._update_Gs(G_smoothing)
        self._g_step(lod, mb, labels_all, rng, G_opt, g_ar, acc=acc)

    # -- live arena ranges: at a given LOD only the layers up to its resolution receive gradients (at the
    # reference schedule's lod 3 a third of each arena).  Zeroing, the finite check and Adam then run over
    # those ranges only; the others hold zero gradient (the whole arenas are zeroed at every LOD change)
    # and zero Adam moments (reset_state at the same points), where Adam would leave the weights
    # unchanged anyway — the trimmed round gives bit-identical weights (tests/test_pg_gan.py).
    _live = None

    def set_lod_live(self, lod):
        if not bool(self._knobs.get('live_ranges', True)):
            self._live = None
            return
        g, d = self.nets.live_names(lod)
        self._live = {id(self.nets.G): self.nets.G.ranges_of(g), id(self.nets.D): self.nets.D.ranges_of(d)}
        if self.nets.gs_moved is not None:
            self.nets.gs_moved |= set(g)

    def _update_Gs(self, beta):
        """The Gs EMA over the G ranges whose Gs may differ from G (every range Adam has stepped since Gs
        was a copy of G: at the reference schedule's lod 3 a third of the arena), or the whole arena (live
        ranges off, a restored state, the CPU)."""
        nets = self.nets
        if self.device.type != 'cuda' or self._live is None or nets.gs_moved is None or not GS_TRIM:
            nets.update_Gs(beta)
            return
        rng = nets.G.ranges_of(sorted(nets.gs_moved))
        tab = self._seg_table(nets.G, rng, key='Gs')
        if tab is not None:
            nets.update_Gs(beta, tab)
        elif len(rng) == 1:
            from rafiki_amd.ops import functional as F
            a, b = rng[0]
            F.lerp_(nets.Gs_master[a:b], nets.G.master[a:b], beta,
                    dst_bf16=None if nets.Gs_bf16 is None else nets.Gs_bf16[a:b])
        else:
            nets.update_Gs(beta)

    def _live_of(self, flat):
        return None if self._live is None else self._live.get(id(flat))

    def _seg_table(self, flat, live, key=None):
        """The cached multi-segment chunk table of ``live`` (None: per-range launches — on the CPU, for
        unaligned ranges, or when the table would have to be built inside a capture)."""
        if self.device.type != 'cuda' or live is None or len(live) < 2:
            return None
        from rafiki_amd.ops import functional as F
        if not F.seg_table_ok(live):
            return None
        tabs = self.__dict__.setdefault('_seg_tables', {})
        key = (id(flat), key, tuple(live))
        tab = tabs.get(key)
        if tab is None and not F._capturing():
            tab = tabs[key] = F.SegTable(self.device, live)
        return tab

    def _zero_grad(self, flat):
        live = self._live_of(flat)
        if live is None:
            _zero(flat.grad)
            return
        tab = self._seg_table(flat, live)
        if tab is not None:
            from rafiki_amd.ops import functional as F
            # the same launch zeroes the step's finite-check flag (the optimizer _finite_guard met last time)
            opt = self.__dict__.get('_opt_of', {}).get(id(flat))
            flag = getattr(opt, 'skip_flag', None)
            F.zero_multi(flat.grad, tab, flag)
            if flag is not None:
                opt._flag_zeroed = True
            return
        for a, b in live:
            _zero(flat.grad[a:b])

    def _finite_guard(self, flat, opt):
        """Set opt.skip_flag when the live gradients hold a non-finite value (pg_gans.py:1180-1191).  Returns
        True when the same launch also advanced the optimizer's step counter (opt.step(bumped=True))."""
        live = self._live_of(flat)
        views = [flat.grad] if live is None else [flat.grad[a:b] for a, b in live]
        if self.device.type == 'cuda':
            from rafiki_amd.engine.flat import FlatAdam
            from rafiki_amd.ops import functional as F
            self.__dict__.setdefault('_opt_of', {})[id(flat)] = opt
            zeroed, opt._flag_zeroed = getattr(opt, '_flag_zeroed', False), False
            tab = self._seg_table(flat, live)
            if tab is not None:
                if not zeroed:
                    F.zero_(opt.skip_flag)
                bump = opt.t if isinstance(opt, FlatAdam) else None
                F.nonfinite_multi(flat.grad, tab, opt.skip_flag, bump=bump)
                return bump is not None
            F.zero_(opt.skip_flag)
            for v in views:
                F.nonfinite_flag(v, opt.skip_flag)
        else:
            opt.skip_flag.fill_(0 if all(bool(torch.isfinite(v).all()) for v in views) else 1)
        return False

    def round_segments(self, lod, mb, level, labels_all, rng, G_opt, D_opt, acc, *, D_repeats=1, G_smoothing=0.99,
                       d_ar=None, g_ar=None, tag=None):
        """train_round as segments for GraphedRounds.run_segments: per D step the gradients ('s': a
        BucketedGrads whose bucket all-reduces start while its backward still runs), the wait for
        those reduces ('e'), then mean + finite guard + Adam + Gs EMA ('g'); likewise the G step.  An
        optimizer segment is merged into the first graph of the next gradient segment.  The reduces
        cover only the buckets the segment's backward wrote (untouched blocks above the current LOD
        are skipped exactly).
        """
        if tag is None:   # plans are per segment shape: never reuse one traced at another LOD / minibatch
            tag = (float(lod), int(mb))
        nets = self.nets

        def d_grads():
            self._d_step(lod, mb, level, labels_all, rng, D_opt, None, apply=False, acc=acc)

        def d_apply():
            d_ar.scale()
            self._apply(nets.D, D_opt, rng)
            self._update_Gs(G_smoothing)

        def g_grads():
            self._g_step(lod, mb, labels_all, rng, G_opt, None, apply=False, acc=acc)

        def g_apply():
            g_ar.scale()
            self._apply(nets.G, G_opt, rng)
            nets.set_requires_grad(nets.d_params, True)

        raw = []
        for r in range(D_repeats):
            d_gr, d_red = d_ar.traced(d_grads, (tag, 'D', r))
            raw += [('s', d_gr), ('e', d_red), ('g', d_apply)]
        g_gr, g_red = g_ar.traced(g_grads, (tag, 'G'))
        raw += [('s', g_gr), ('e', g_red), ('g', g_apply)]
        segs = []
        for kind, fn in raw:
            if segs and kind in ('g', 's') and segs[-1][0] == 'g':
                prev = segs.pop()[1]
                if kind == 's':
                    fn.pre.append(prev)   # the previous step's optimizer runs in the first graph of this one
                    segs.append((kind, fn))
                else:
                    segs.append(('g', (lambda a, b: (lambda: (a(), b())))(prev, fn)))
            else:
                segs.append((kind, fn))
        return segs

    def _apply(self, flat, opt, rng):
        bumped = self._finite_guard(flat, opt)
        # the multi-segment Adam launch also advances the random stream's step counter (else its own launch)
        bump = rng.step if self.device.type == 'cuda' and isinstance(getattr(rng, 'step', None), torch.Tensor) \
            else None
        if not opt.step(live=self._live_of(flat), bumped=bumped, bump=bump):
            rng.advance()

    def _fused_loss(self, grads=None):
        """The fused WGAN loss head (WganLossFn) applies: fp32 on the GPU, no label logits."""
        return (self.device.type == 'cuda' and self.nets.label_size == 0 and self.nets.act_dtype == torch.float32
                and (grads is None or grads.dtype == torch.float32))

    def _one(self):
        """A resident scalar 1.0: the backward seed of a scalar loss (no ones_like kernel per step)."""
        one = self.__dict__.get('_one_t')
        if one is None:
            one = self._one_t = torch.ones((), device=self.device)
        return one

    def _score_seed(self, n, ld):
        """Constant [n, ld] fp32 rows with 1 in column 0: the input-gradient seed of sum(scores) taken on
        the raw discriminator output (no slice / select backward kernels)."""
        key = (n, ld)
        seeds = self.__dict__.setdefault('_seeds', {})
        if key not in seeds:
            t = torch.zeros((n, ld), device=self.device)
            t[:, 0] = 1.0
            seeds[key] = t
        return seeds[key]

    def _d_step(self, lod, mb, level, labels_all, rng, opt, ar, wgan_lambda=10.0, wgan_epsilon=0.001,
                wgan_target=1.0, apply=True, acc=None):
        """_D_wgangp_acgan (pg_gans.py:1291-1328) + D optimizer step (``apply=False``: gradients only).
        acc[:4] += the step's mean (loss, real score, fake score, |grad|).  The weights' Winograd / X6-plane
        forms are derived once per step (A.cached_weight_transforms), not once per conv call."""
        with A.cached_weight_transforms(self._cacheable()):
            stats = self._d_grads(lod, mb, level, labels_all, rng, ar, wgan_lambda, wgan_epsilon, wgan_target, acc)
        if apply:
            self._apply(self.nets.D, opt, rng)
        if stats is not None and acc is not None:
            acc[:4] += stats
        return stats

    def _cacheable(self):
        nets = self.nets
        return list(nets.d_params.values()) + list(nets.g_params.values()) if self.device.type == 'cuda' else []

    def _d_grads(self, lod, mb, level, labels_all, rng, ar, wgan_lambda, wgan_epsilon, wgan_target, acc):
        nets = self.nets
        PG, PD = nets.src_G(), nets.src_D()
        nets.set_requires_grad(nets.g_params, False)
        nets.set_requires_grad(nets.d_params, True)
        self._zero_grad(nets.D)
        idx = self._shard(rng.randint(level.shape[0], mb * self.world, TrialRng.D_IDX)).to(level.device)
        reals = self._reals(level, idx, lod - math.floor(lod))
        labels = labels_all.index_select(0, idx) if nets.label_size else torch.zeros((mb, 0), device=self.device)
        with torch.no_grad():
            fakes = nets.generator(PG, self._latents(mb, rng, TrialRng.D_LAT), labels, lod)
        fused = self._fused_loss()
        alpha = self._shard(rng.rand((mb * self.world, 1, 1, 1), TrialRng.D_ALPHA))
        if fused and reals.dtype == torch.float32 and fakes.dtype == torch.float32 and reals[0].numel() % 4 == 0:
            # [reals; fakes] and the interpolates in one native pass
            rf_in = torch.empty((2 * mb,) + tuple(reals.shape[1:]), device=reals.device, dtype=torch.float32)
            mixed = torch.empty_like(reals)
            _lib.call("rk_wgan_mix", S._p(reals.contiguous()), S._p(fakes.contiguous()), S._p(alpha.contiguous()),
                      S._p(rf_in), S._p(mixed), mb, reals[0].numel(), S._s())
            mixed.requires_grad_(True)
        else:
            rf_in = torch.cat([reals, fakes.to(reals.dtype)], 0)
            mixed = torch.lerp(reals.float(), fakes.float(), alpha).to(reals.dtype).detach().requires_grad_(True)
        # real and fake minibatches share one batched D evaluation (2 independent mbstd segments):
        # half the launches, twice the GEMM rows, one weight-gradient contribution instead of two
        rf = nets.discriminator(PD, rf_in, lod, segs=2, raw=fused)
        if fused:
            mixed_raw = nets.discriminator(PD, mixed, lod, raw=True)
            if ar is not None:
                ar.begin()
            (grads,) = torch.autograd.grad(mixed_raw, mixed, self._score_seed(*mixed_raw.shape), create_graph=True)
            loss = WganLossFn.apply(rf, grads, wgan_lambda / wgan_target ** 2, wgan_target, wgan_epsilon,
                                    None if acc is None else acc[0:4])
            stats = None
        else:
            rf_s, rf_l = rf
            real_s, fake_s = rf_s[:mb], rf_s[mb:]
            real_l, fake_l = rf_l[:mb], rf_l[mb:]
            loss = fake_s - real_s
            mixed_s, _ = nets.discriminator(PD, mixed, lod)
            if ar is not None:
                ar.begin()
            (grads,) = torch.autograd.grad(mixed_s.sum(), mixed, create_graph=True)
            penalty, norms = _GradPenaltyFn.apply(grads, wgan_lambda / wgan_target ** 2, wgan_target)
            loss = torch.addcmul(loss + penalty, real_s, real_s, value=wgan_epsilon)
            if nets.label_size:
                loss = loss + _softmax_xent(real_l, labels) + _softmax_xent(fake_l, labels)
            stats = torch.stack([loss.detach(), real_s.detach(), fake_s.detach(), norms.detach()]).mean(1)
            loss = loss.mean()
        # data-parallel rounds launch their all-reduce buckets from post-accumulate-grad hooks, so
        # they keep autograd's accumulation
        with A.accumulate_weight_grads_in_place(nets.d_params.values()) if ar is None else contextlib.nullcontext():
            loss.backward(self._one() if loss.is_cuda else None)
        if ar is not None:
            ar.finish()
        return stats

    def _g_step(self, lod, mb, labels_all, rng, opt, ar, apply=True, acc=None):
        """_G_wgan_acgan (pg_gans.py:1276-1289) + G optimizer step (``apply=False``: gradients only).
        acc[4] += the step's mean loss."""
        with A.cached_weight_transforms(self._cacheable()):
            stat = self._g_grads(lod, mb, labels_all, rng, ar, acc)
        if apply:
            self._apply(self.nets.G, opt, rng)
            self.nets.set_requires_grad(self.nets.d_params, True)
        if stat is not None and acc is not None:
            acc[4] += stat
        return stat

    def _g_grads(self, lod, mb, labels_all, rng, ar, acc):
        nets = self.nets
        PG, PD = nets.src_G(), nets.src_D()
        nets.set_requires_grad(nets.d_params, False)
        nets.set_requires_grad(nets.g_params, True)
        self._zero_grad(nets.G)
        labels = self._rand_labels(labels_all, mb, rng)
        fakes = nets.generator(PG, self._latents(mb, rng, TrialRng.G_LAT), labels, lod)
        if self._fused_loss():
            out = nets.discriminator(PD, fakes, lod, raw=True)
            loss = WganLossFn.apply(out, None, 0.0, 0.0, 0.0, None if acc is None else acc[4:5])
            stat = None
        else:
            fake_s, fake_l = nets.discriminator(PD, fakes, lod)
            loss = -fake_s
            if nets.label_size:
                loss = loss + _softmax_xent(fake_l, labels)
            loss = loss.mean()
            stat = loss.detach()
        if ar is not None:
            ar.begin()
        # data-parallel rounds launch their all-reduce buckets from post-accumulate-grad hooks, so
        # they keep autograd's accumulation
        with A.accumulate_weight_grads_in_place(nets.g_params.values()) if ar is None else contextlib.nullcontext():
            loss.backward(self._one() if loss.is_cuda else None)
        if ar is not None:
            ar.finish()
        return stat

    # ------------------------------------------------------------------ generation
    @torch.no_grad()
    def generate(self, n, seed=1000, batch=256, use_Gs=True):
        """n images uint8 NHWC [n, R, R, C] at full resolution (pg_gans.py:124-136 / Network.run:
        out_mul=127.5, out_add=127.5, nearest upscale of lower-LOD output).

        In a data-parallel trial every rank draws the same latents and renders only its slice of each
        batch; an all-gather assembles the batch on every rank (the reference splits Network.run over
        num_gpus towers, pg_gans.py:691-711)."""
        nets = self.nets
        P = nets.src_Gs() if use_Gs else nets.src_G()
        lod = float(self.lod or 0.0)
        g = torch.Generator(device=self.device)
        g.manual_seed(int(seed))
        world, rank = self.world, self.rank
        shard = world > 1 and torch.distributed.is_available() and torch.distributed.is_initialized()
        outs = []
        for b in range(0, n, batch):
            m = min(batch, n - b)
            lat = torch.randn((m, nets.latent_size), generator=g, device=self.device)
            lab = torch.zeros((m, nets.label_size), device=self.device)
            if nets.label_size:
                lab[torch.arange(m), torch.randint(0, nets.label_size, (m,), generator=g, device=self.device)] = 1.0
            lo, hi = 0, m
            if shard:
                per = -(-m // world)
                lo, hi = min(m, rank * per), min(m, (rank + 1) * per)
            with torch.no_grad():
                img = self._slice_images(nets.generator(P, lat[lo:hi], lab[lo:hi], lod)).float()
            factor = nets.resolution // img.shape[1]
            if factor > 1:
                img = A.upscale2d(img, factor)
            u8 = (img * 127.5 + 127.5).round().clamp(0, 255).to(torch.uint8)
            if shard:
                u8 = self._gather_rows(u8, per, m)
            outs.append(u8.cpu())
        return torch.cat(outs).numpy()

    def _gather_rows(self, part, per, m):
        """Concatenate every rank's rows (``per`` each, the last ranks may hold fewer) -> [m, ...]."""
        import torch.distributed as dist
        comm = torch.device('cuda', self.ctx.dist.local_rank) if self.ctx.dist.backend == 'nccl' else torch.device('cpu')
        buf = torch.zeros((per,) + tuple(part.shape[1:]), dtype=part.dtype, device=comm)
        buf[:part.shape[0]] = part.to(comm)
        bufs = [torch.empty_like(buf) for _ in range(self.world)]
        dist.all_gather(bufs, buf)
        return torch.cat(bufs)[:m]

    # ------------------------------------------------------------------ evaluate
    def evaluate(self, dataset_uri):
        n = int(self._knobs.get('eval_images', 10000))
        ds = load_gan_dataset(dataset_uri)
        real = ds.images[0]  # [N, C, R, R]
        labels = getattr(ds, 'class_labels', None)
        if labels is None and ds.labels.shape[1] > 0:
            labels = ds.labels.argmax(1)
        if labels is None:
            labels = _kmeans_labels(real, k=10, seed=0)
        clf = _train_eval_classifier(real, labels, self.device,
                                     epochs=int(self._knobs.get('eval_classifier_epochs', 3)))
        fake = self.generate(n, seed=int(self._knobs.get('eval_seed', 1)))
        probs = _classify(clf, fake)
        return float(_inception_score(probs, splits=10))

    # ------------------------------------------------------------------ predict
    def predict(self, queries):
        """queries = [grid_w, grid_h, n_images] (pg_gans.py:166-214) -> list of JPEG paths; a list of
        such triples -> a list of path lists."""
        if len(queries) and isinstance(queries[0], (list, tuple)):
            return [self._predict_one(q) for q in queries]
        return self._predict_one(queries)

    def _predict_one(self, q):
        from PIL import Image
        gw, gh, num = int(q[0]), int(q[1]), int(q[2])
        out_dir = os.environ.get('RAFIKI_OUTPUT_DIR') or os.path.join(tempfile.gettempdir(), 'rafiki_pg_gan')
        out_dir = os.path.join(out_dir, uuid.uuid4().hex[:12])
        os.makedirs(out_dir, exist_ok=True)
        rs = np.random.RandomState(1000)
        paths = []
        for i in range(num):
            cnt = gw * gh
            imgs = self.generate(cnt, seed=int(rs.randint(1 << 30)))  # [cnt, R, R, C]
            R, C = imgs.shape[1], imgs.shape[3]
            grid_w = max(int(np.ceil(np.sqrt(cnt))), 1)
            grid_h = max((cnt - 1) // grid_w + 1, 1)
            grid = np.zeros((grid_h * R, grid_w * R, C), np.uint8)
            for j in range(cnt):
                x, y = (j % grid_w) * R, (j // grid_w) * R
                grid[y:y + R, x:x + R] = imgs[j]
            im = Image.fromarray(grid[..., 0], 'L') if C == 1 else Image.fromarray(grid, 'RGB')
            p = os.path.abspath(os.path.join(out_dir, 'output%d.jpeg' % i))
            im.save(p, 'JPEG')
            paths.append(p)
        return paths

    # ------------------------------------------------------------------ params
    def dump_parameters(self):
        st = self.nets.state()
        return {'G': pickle.dumps(st['G'], protocol=pickle.HIGHEST_PROTOCOL),
                'D': pickle.dumps(st['D'], protocol=pickle.HIGHEST_PROTOCOL),
                'Gs': pickle.dumps(st['Gs'], protocol=pickle.HIGHEST_PROTOCOL),
                'meta': dict(self._meta, lod=float(self.lod or 0.0))}

    def load_parameters(self, params):
        meta = dict(params['meta'])
        self.lod = float(meta.pop('lod', 0.0))
        self._meta = meta
        self.nets = PgNetworks(device=self.device, seed=self.seed, **meta)
        self.nets.load_state({k: pickle.loads(params[k]) for k in ('G', 'D', 'Gs')})

    def destroy(self):
        from ..ops.graphs import quiesced
        with quiesced():
            self.graphs = None
            self.nets = None


# ============================================================================== eval helpers
class _GradPenaltyFn(torch.autograd.Function):
    """WGAN-GP penalty of per-sample gradients g [mb, ...]: -> (lambda (|g| - t)^2 [mb], |g| [mb]).  Forward:
    one norm reduction; backward: one broadcast multiply, d/dg = 2 lambda (|g| - t) / |g| * g * gout (the
    autograd chain of square / sum / sqrt / sub / square / mul was ~14 small kernels per D step)."""

    @staticmethod
    def forward(ctx, g, lam, target):
        n = torch.linalg.vector_norm((g if g.dtype == torch.float64 else g.float()).reshape(g.shape[0], -1), dim=1)
        ctx.save_for_backward(g, n)
        ctx.lam, ctx.target = lam, target
        return (n - target).square() * lam, n

    @staticmethod
    def backward(ctx, gp, gn):
        g, n = ctx.saved_tensors
        coef = gp * (2.0 * ctx.lam) * (n - ctx.target) / n.clamp_min(1e-30)
        if gn is not None:
            coef = coef + gn / n.clamp_min(1e-30)
        return (g * coef.view((-1,) + (1,) * (g.dim() - 1)).to(g.dtype)), None, None


def _zero(t):
    if t.is_cuda:
        from rafiki_amd.ops import functional as F
        return F.zero_(t)
    return t.zero_()


class WganLossFn(torch.autograd.Function):
    """The label-free WGAN losses as one fused head on the raw discriminator output (pgg wgan kernels,
    csrc/kernels/pggan.hip):
      D (``g`` given): mean_r [fake_r - real_r + lam (|g_r| - t)^2 + eps real_r^2]  (pg_gans.py:1291-1315)
        with real / fake = column 0 of rows r / mb + r of ``s`` and g_r the penalty gradient rows;
      G (``g`` None):  mean_r [-s_r]                                               (pg_gans.py:1276-1289).
    ``acc`` (optional fp32, 4 resp. 1 elements) += the means (loss, real, fake, |g|) on the device.
    Backward: d/ds (zeros off column 0) and d/dg = 2 lam (|g| - t) / |g| g / mb, one kernel."""

    @staticmethod
    def forward(ctx, s, g, lam, target, eps, acc):
        s = s.contiguous()
        ld = s.shape[1]
        if g is not None:
            g = g.contiguous()
            mb, P = g.shape[0], g.numel() // g.shape[0]
            assert s.shape[0] == 2 * mb and g.dtype == torch.float32
        else:
            mb, P = s.shape[0], 0
        assert s.dtype == torch.float32 and (acc is None or (acc.dtype == torch.float32 and acc.is_contiguous()))
        rows = torch.empty((4, mb), device=s.device, dtype=torch.float32)
        loss = torch.empty((), device=s.device, dtype=torch.float32)
        _lib.call("rk_wgan_loss_fwd", S._p(s), ld, mb, S._p(g), P, float(lam), float(target), float(eps),
                  S._p(rows), S._p(loss), S._p(acc), S._s())
        ctx.save_for_backward(s, g, rows)
        ctx.k = (ld, mb, P, float(lam), float(target), float(eps))
        return loss

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gl):
        s, g, rows = ctx.saved_tensors
        ld, mb, P, lam, target, eps = ctx.k
        ds = torch.empty_like(s)
        dg = torch.empty_like(g) if g is not None else None
        _lib.call("rk_wgan_loss_bwd", S._p(gl.float().contiguous()), S._p(s), ld, mb, S._p(g), P, lam, target, eps,
                  S._p(rows), S._p(ds), S._p(dg), S._s())
        return ds, (dg.view(g.shape) if dg is not None else None), None, None, None, None


def _softmax_xent(logits, onehot):
    return -(torch.log_softmax(logits.float(), 1) * onehot).sum(1)


def _inception_score(probs, splits=10, eps=1e-12):
    probs = np.asarray(probs, dtype=np.float64)
    scores = []
    n = probs.shape[0]
    for i in range(splits):
        part = probs[i * n // splits:(i + 1) * n // splits]
        if len(part) == 0:
            continue
        py = part.mean(0, keepdims=True)
        kl = (part * (np.log(part + eps) - np.log(py + eps))).sum(1).mean()
        scores.append(np.exp(kl))
    return float(np.mean(scores))


def _kmeans_labels(real, k=10, seed=0, fit_max=20000):
    """Pseudo-classes for unlabeled evaluation sets: k-means on 8x8 box-filtered images."""
    from sklearn.cluster import KMeans
    x = real.astype(np.float32)
    N, C, R, _ = x.shape
    f = max(1, R // 8)
    x = x.reshape(N, C, R // f, f, R // f, f).mean((3, 5)).reshape(N, -1)
    km = KMeans(n_clusters=min(k, max(2, N // 4)), n_init=3, random_state=seed).fit(x[:fit_max])
    return km.predict(x)


def _train_eval_classifier(real, labels, device, epochs=3):
    from rafiki_amd.engine.convnet import ConvNetEngine
    N, C, R, _ = real.shape
    ncls = int(np.max(labels)) + 1
    eng = ConvNetEngine(num_classes=max(ncls, 2), in_channels=C, image_size=R, cfg=(32, 'M', 64, 'M', 128, 'M'),
                        fc_dims=(128,), device=device, seed=0, optimizer='adam', lr=2e-3, weight_decay=0.0)
    imgs = real.transpose(0, 2, 3, 1)
    x_all = eng.prepare_inputs(imgs)
    y_all = torch.as_tensor(np.asarray(labels), dtype=torch.int32, device=eng.device)
    bs = min(128, N)
    g = torch.Generator().manual_seed(0)
    for _ in range(max(1, epochs)):
        perm = torch.randperm(N, generator=g).to(eng.device)
        for b in range(0, N - bs + 1, bs):
            idx = perm[b:b + bs]
            eng.train_step(x_all.index_select(0, idx), y_all.index_select(0, idx))
    eng.prepare_eval()
    return eng


def _classify(eng, imgs_nhwc, batch=512):
    out = []
    for b in range(0, len(imgs_nhwc), batch):
        x = eng.prepare_inputs(imgs_nhwc[b:b + batch])
        out.append(eng.forward_eval(x).float().cpu().numpy())
    return np.concatenate(out)


if __name__ == '__main__':
    from rafiki_amd.model import test_model_class
    test_model_class(__file__, 'PgGan', TaskType.IMAGE_GENERATION, {},
                     'synthetic://image?n=512&size=16&channels=1&classes=4&seed=0',
                     'synthetic://image?n=256&size=16&channels=1&classes=4&seed=1',
                     queries=[[2, 2, 1]],
                     knobs={'D_repeats': 1, 'minibatch_base': 4, 'G_lrate': 1e-3, 'D_lrate': 1e-3,
                            'lod_initial_resolution': 4, 'total_kimg': 0.5, 'lod_training_kimg': 0.2,
                            'lod_transition_kimg': 0.2, 'fmap_base': 256, 'fmap_max': 64, 'eval_images': 256})
