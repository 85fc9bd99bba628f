"""Shared machinery for the native image-classification models (VGG-small, FeedForward MLP).

A trial uploads its whole train split to HBM once (uint8 -> packed fp32 / bf16 NHWC by one gfx950 kernel),
captures the training step into a hipGraph and replays it per batch; shuffling and batching are
device-side index_selects.  evaluate/predict use hipGraph-captured forwards per batch bucket.
Task I/O contract (reference docs/src/user/tasks.rst:23-63): a query is an HxW (grayscale) or
HxWxC image as nested lists; a prediction is the list of class probabilities.
"""
from __future__ import annotations

import base64
import io
import math
import pickle
import time

import numpy as np
import torch

from ..engine.convnet import ConvNetEngine, default_dtype
from ..engine.flat import FlatSGD
from ..model import BaseModel, dataset_utils, logger
from ..parallel.context import current as trial_context
from ..ops.graphs import device_sync
from ..utils import faults


class NativeImageClassifier(BaseModel):
    """Subclasses define ``_engine_kwargs()`` and their knob config."""

    DEFAULT_IMAGE_SIZE = 32

    def __init__(self, **knobs):
        super().__init__(**knobs)
        self._knobs = dict(knobs)
        self._engine = None
        self._meta = {}
        self.device = trial_context().device

    # --------------------------------------------------------------------- subclass hooks
    def _engine_kwargs(self, num_classes, channels, image_size):
        raise NotImplementedError

    @property
    def image_size(self):
        return int(self._knobs.get('image_size', self.DEFAULT_IMAGE_SIZE))

    # ------------------------------------------------------------------------ data helpers
    def _load(self, uri):
        ds = dataset_utils.load_dataset_of_image_files(uri, image_size=self.image_size)
        images, labels = ds.as_arrays()
        if images.shape[1] != self.image_size or images.shape[2] != self.image_size:
            images = dataset_utils.resize_as_images(images, self.image_size)
        return images, labels, ds.classes

    def _build(self, num_classes, channels, dtype=None):
        kw = self._engine_kwargs(num_classes, channels, self.image_size)
        # compute dtype: fp32 (reference precision) unless the trial / RAFIKI_DTYPE opts into bf16
        kw.setdefault('dtype', dtype or self._knobs.get('dtype') or default_dtype())
        self._engine = ConvNetEngine(num_classes=num_classes, in_channels=channels, image_size=self.image_size,
                                     device=self.device, seed=int(self._knobs.get('seed', 0)), **kw)
        self._meta = {'num_classes': num_classes, 'channels': channels, 'image_size': self.image_size,
                      'dtype': self._engine.dtype}

    # ------------------------------------------------------------------------ BaseModel API
    def train(self, dataset_uri):
        tm = self.timings = {}
        t_start = time.perf_counter()
        images, labels, classes = self._load(dataset_uri)
        tm['load'] = time.perf_counter() - t_start
        channels = 1 if images.ndim == 3 else images.shape[-1]
        self._build(max(classes, 2), channels)
        tm['build'] = time.perf_counter() - t_start - tm['load']
        eng = self._engine
        x_all = eng.prepare_inputs(images)
        y_all = torch.from_numpy(np.asarray(labels, dtype=np.int32)).to(eng.device)  # (cached arrays are read-only)
        tm['upload'] = time.perf_counter() - t_start - tm['load'] - tm['build']
        n = x_all.shape[0]
        bs = int(min(self._knobs.get('batch_size', 128), n))
        epochs = float(self._knobs.get('epochs', 1))
        steps_per_epoch = max(1, n // bs)
        total = max(1, int(math.ceil(epochs * steps_per_epoch)))
        use_graph = eng.device.type == 'cuda'
        t_cap = time.perf_counter()
        # one graph per step that also gathers its minibatch by a device-side counter from a per-epoch
        # index schedule and reads its LR multiplier from a per-step table: a replay per step, no copies
        scheduled = use_graph and isinstance(eng.opt, FlatSGD)
        if scheduled:
            eng.capture_scheduled(x_all, y_all, steps_per_epoch, bs)
        elif use_graph:
            eng.capture(bs)
        tm['capture'] = time.perf_counter() - t_cap
        xb = torch.empty(eng.input_shape(bs), dtype=x_all.dtype, device=eng.device)
        yb = torch.empty((bs,), dtype=torch.int32, device=eng.device)
        gen = torch.Generator(device=eng.device) if eng.device.type == 'cuda' else torch.Generator()
        gen.manual_seed(int(self._knobs.get('seed', 0)))
        logger.define_loss_plot()
        logger.define_plot('Train accuracy', ['train_acc'], x_axis='epoch')
        logger.define_plot('Throughput', ['images_per_sec'], x_axis='epoch')
        sched = self._knobs.get('lr_schedule', 'cosine')
        ctx = trial_context()
        ck = ctx.checkpoint
        step = 0
        epoch = 0
        if ck is not None:
            saved = ck.load()
            if saved is not None:
                self._restore_ckpt(saved['state'], gen)
                step, epoch = int(saved['state']['step']), int(saved['epoch']) + 1
                logger.log('resumed from checkpoint after epoch {} (step {})'.format(saved['epoch'], step))
        t_loop = time.perf_counter()
        while step < total:
            perm = torch.randperm(n, device=eng.device, generator=gen)
            eng.reset_metrics()
            t0 = time.perf_counter()
            done = 0
            if scheduled:
                cosine = hasattr(eng.opt, 'set_lr_scale') and sched == 'cosine'
                lrs = [0.5 * (1.0 + math.cos(math.pi * (step + b) / total)) if cosine else 1.0
                       for b in range(steps_per_epoch)]
                eng.set_schedule(perm[:steps_per_epoch * bs].view(steps_per_epoch, bs), lr_scales=lrs)
            for b in range(steps_per_epoch):
                if step >= total:
                    break
                faults.maybe_fail('train_step', step=step, rank=ctx.rank)
                if scheduled:
                    eng.replay()
                    step += 1
                    done += 1
                    continue
                if hasattr(eng.opt, 'set_lr_scale') and sched == 'cosine':
                    eng.opt.set_lr_scale(0.5 * (1.0 + math.cos(math.pi * step / total)))
                idx = perm[b * bs:(b + 1) * bs]
                torch.index_select(x_all, 0, idx, out=xb)
                torch.index_select(y_all, 0, idx, out=yb)
                if use_graph:
                    eng.step_graph(xb, yb)
                else:
                    eng.train_step(xb, yb)
                step += 1
                done += 1
            seen = max(1, int(eng.seen.item()))  # host sync once per epoch
            dt = max(1e-9, time.perf_counter() - t0)
            logger.log_loss(loss=float(eng.loss_sum.item()) / seen, epoch=epoch)
            logger.log(train_acc=float(eng.correct.item()) / seen, epoch=epoch)
            logger.log(images_per_sec=done * bs / dt, epoch=epoch)
            if ck is not None and ck.due(epoch) and step < total:
                ck.save(self._ckpt_state(step, gen), epoch)
            faults.maybe_fail('crash', epoch=epoch, rank=ctx.rank)
            epoch += 1
        if eng.device.type == 'cuda':
            device_sync(eng.device)
        tm['loop'] = time.perf_counter() - t_loop
        if eng.device.type == 'cuda':
            logger.log(hbm_peak_bytes=int(torch.cuda.max_memory_allocated(eng.device)))
        t_pe = time.perf_counter()
        eng.prepare_eval()
        tm['prepare_eval'] = time.perf_counter() - t_pe
        tm['total'] = time.perf_counter() - t_start
        self.timings = {k: round(v, 4) for k, v in tm.items()}

    # ----------------------------------------------------------------- checkpoint / resume
    def _ckpt_state(self, step, gen):
        eng = self._engine
        opt = [t.detach().cpu().numpy().copy() for t in eng._opt_tensors()]
        return {'step': int(step), 'master': eng.flat.master.detach().cpu().numpy().copy(),
                'running': eng.running.detach().cpu().numpy().copy(), 'opt': opt,
                'gen': gen.get_state().numpy().copy(), 'meta': dict(self._meta)}

    def _restore_ckpt(self, st, gen):
        eng = self._engine
        eng.flat.master.copy_(torch.as_tensor(st['master']))
        eng.flat.sync_bf16()
        eng.running.copy_(torch.as_tensor(st['running']))
        for t, v in zip(eng._opt_tensors(), st['opt']):
            t.copy_(torch.as_tensor(v))
        gen.set_state(torch.as_tensor(st['gen']))

    def _probs(self, images_uint8):
        eng = self._engine
        out = []
        chunk = 4096
        for i in range(0, len(images_uint8), chunk):
            x = eng.prepare_inputs(images_uint8[i:i + chunk])
            out.append(eng.forward_eval_graphed(x).clone() if eng.device.type == 'cuda' else eng.forward_eval(x))
        return torch.cat(out) if out else torch.zeros((0, self._meta['num_classes']))

    def evaluate(self, dataset_uri):
        images, labels, _ = self._load(dataset_uri)
        probs = self._probs(images)
        pred = probs.argmax(1).cpu().numpy()
        return float((pred == np.asarray(labels)).mean())

    def _queries_to_images(self, queries):
        from .. import runtime
        # nested-list queries (the JSON query format) through the native walker (~10x numpy)
        arr = runtime.pylist_u8(queries) if isinstance(queries, (list, tuple)) else None
        if arr is None:
            arr = np.asarray(queries)
        if arr.dtype != np.uint8:
            arr = np.clip(arr, 0, 255).astype(np.uint8)
        if arr.ndim == 2:
            arr = arr[None]
        if arr.shape[1] != self.image_size or arr.shape[2] != self.image_size:
            arr = dataset_utils.resize_as_images(arr, self.image_size)
        ch = self._meta['channels']
        if ch == 1 and arr.ndim == 4:
            arr = arr.mean(-1).astype(np.uint8)
        if ch > 1 and arr.ndim == 3:
            arr = np.repeat(arr[..., None], ch, -1)
        return arr

    def input_signature(self):
        """Models with equal signatures accept the same uint8 image batch (the predictor converts and
        uploads a request once per signature, not once per model)."""
        return ('image_u8', self.image_size, self._meta['channels'])

    def queries_to_images(self, queries):
        return self._queries_to_images(queries)

    def predict_proba_images(self, images) -> torch.Tensor:
        """uint8 [Q, H, W(, C)] (host or device) at this model's size -> device probabilities [Q, C]."""
        return self._probs(images)

    @property
    def num_classes(self):
        return int(self._meta['num_classes'])

    def serving_engine(self):
        """The trained engine (the predictor groups same-architecture engines into one network)."""
        return self._engine

    def release_training(self):
        """Keep only the inference state (trainer -> predictor HBM handoff, predictor.resident)."""
        if self._engine is not None:
            self._engine.release_training()

    def prepare_serving(self):
        """Fold BN into inference coefficients ahead of a graph capture (forward_into is capture-safe)."""
        if self._engine._eval_coeffs is None:
            self._engine.prepare_eval()

    def forward_into(self, images_dev, out):
        """uint8 device batch [Q, H, W(, C)] -> probabilities written into ``out`` [Q, C] fp32: the
        pack kernel + the un-graphed eval forward, so a caller can capture it inside a larger graph
        (the predictor's one-graph-per-bucket ensemble)."""
        eng = self._engine
        return eng._forward_eval_gpu(eng.prepare_inputs(images_dev), out)

    def predict_proba(self, queries) -> torch.Tensor:
        """Device tensor [Q, num_classes] (used by the predictor's on-device ensemble)."""
        return self._probs(self._queries_to_images(queries))

    def predict(self, queries):
        if len(queries) == 0:
            return []
        return self.predict_proba(queries).float().cpu().tolist()

    def dump_parameters(self):
        return {'meta': dict(self._meta), 'state': self._engine.state_dict(), 'knobs': dict(self._knobs)}

    def load_parameters(self, params):
        meta = params['meta']
        self._build(meta['num_classes'], meta['channels'], dtype=meta.get('dtype', 'bf16'))
        self._engine.load_state_dict(params['state'])
        self._engine.prepare_eval()

    def resident_bytes(self):
        return self._engine.resident_bytes() if self._engine is not None else 0

    def destroy(self):
        from ..ops.graphs import quiesced
        with quiesced():   # the engine's captured graphs die here
            self._engine = None
