"""Native BiLSTM tagger training step (PyBiLstm on the GPU).

Reference: examples/models/pos_tagging/PyBiLstm.py:185-235 (train loop: Adam, cross-entropy over the
padded batch), :249-268 (Embedding(V, E, padding_idx=0) -> Dropout -> BiLSTM(E, H) -> Linear(2H, tags)).

Every kernel of a step is in-tree (csrc/kernels): embedding gather fused with the Philox dropout mask
(tagger.hip), the input projection / output layer / all weight and data gradients on ``sgemm`` (f32.py
linear, linear_dx, linear_dw, colsum), the recurrence forward and BPTT as one persistent launch each
(lstm.hip), softmax cross-entropy with ignore_index and a device 1/#tokens scale (loss_optim.hip),
the embedding gradient as ordered run sums over host-sorted ids (tagger.hip), and one Adam launch
over a flat parameter arena (loss_optim.hip).

Layout: every extent is zero-padded once, in the arena, so any knob value stays on the in-tree
kernels — E and the tag count to multiples of 4 (16-B GEMM rows), the hidden size per gate block to
HP in {64, 128} (the recurrence kernels' tiles).  Padded rows / columns start at zero, receive
exactly zero gradient (zero activations in, zero upstream gradient out) and so stay zero under Adam:
the arena trains exactly the unpadded model.  nn.LSTM's two bias vectors are kept as two parameters
(each gets the full bias gradient), as torch's Adam sees them.

A step of a batch shape (L, B) is captured into a hipGraph the first time that shape is seen (after
an eager run that autotunes its GEMMs) and replayed afterwards; sentences are bucketed by length, so
the number of distinct shapes is the number of distinct bucket lengths.  Per step the host packs ids,
labels, the embedding-gradient runs and 1/#tokens into one int32 buffer and sends it with a single
async copy from pinned memory (double-buffered, so packing batch k+1 overlaps step k on the GPU).
The device step counter drives both Adam's bias corrections and the dropout stream, so replays draw
fresh masks.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from ..ops import _lib
from ..ops import f32 as S
from ..ops import graphs
from ..ops.functional import _p, _s

IGNORE = -100
_DROP_STREAM = 0x7a67   # Philox stream id of the tagger's dropout


def _cdiv(a: int, b: int) -> int:
    return -(-a // b)


def pack_batch(x_bl: np.ndarray, y_bl, padding_idx: int = 0, vocab: Optional[int] = None) -> np.ndarray:
    """One batch as the int32 words the step reads: x_bl / y_bl are [B, L] (batch-first, like the
    reference's batches; labels IGNORE where no token).  Layout, with n = L*B tokens in time-major
    order (t, b): [ids n | labels n | perm n | run ids n | run starts n+1 | #runs | 1/#labelled as
    float bits].  perm is the stable argsort of the ids; run u covers perm[start[u]:start[u+1]] and
    has id uniq[u] (-1 for the padding id: no gradient).  With ``vocab``, ids outside [0, vocab) become
    the padding id, as the forward's gather treats them (no gradient row is written for them)."""
    B, L = x_bl.shape
    n = B * L
    ids = np.ascontiguousarray(x_bl.T, dtype=np.int32).reshape(-1)
    if vocab is not None:
        ids = np.where((ids < 0) | (ids >= vocab), np.int32(padding_idx), ids)
    if y_bl is None:
        labels = np.full(n, IGNORE, np.int32)
    else:
        labels = np.ascontiguousarray(y_bl.T, dtype=np.int32).reshape(-1)
    perm = np.argsort(ids, kind='stable').astype(np.int32)
    s = ids[perm]
    starts = np.flatnonzero(np.diff(s)) + 1 if n > 1 else np.zeros(0, np.int64)
    starts = np.concatenate(([0], starts, [n])).astype(np.int32)
    uniq = s[starts[:-1]].astype(np.int32)
    uniq[uniq == padding_idx] = -1
    U = len(uniq)
    cnt = int((labels != IGNORE).sum())
    out = np.zeros(5 * n + 3, np.int32)
    out[0:n] = ids
    out[n:2 * n] = labels
    out[2 * n:3 * n] = perm
    out[3 * n:3 * n + U] = uniq
    out[4 * n:4 * n + U + 1] = starts
    out[5 * n + 1] = U
    out[5 * n + 2:5 * n + 3] = np.array([1.0 / max(1, cnt)], np.float32).view(np.int32)
    return out


class TaggerEngine:
    """Flat padded parameters + Adam state of one PyBiLstm ``Net`` (attributes emb, lstm, out), and its
    training step on the in-tree kernels.  ``step`` takes batch-first numpy ids / labels."""

    def __init__(self, net, lr: float, dropout: float, *, seed: int = 0, betas=(0.9, 0.999), eps=1e-8):
        dev = net.emb.weight.device
        assert dev.type == 'cuda', 'TaggerEngine runs on the GPU kernels'
        V, E = net.emb.weight.shape
        H = net.lstm.hidden_size
        NT = net.out.out_features
        if H > 128 or net.lstm.num_layers != 1 or not net.lstm.bidirectional:
            raise ValueError('TaggerEngine: one bidirectional layer of hidden <= 128 (got {})'.format(H))
        self.V, self.E, self.H, self.NT = V, E, H, NT
        self.EP, self.HP, self.NTP = _cdiv(E, 4) * 4, (64 if H <= 64 else 128), _cdiv(NT, 4) * 4
        self.padding_idx = net.emb.padding_idx if net.emb.padding_idx is not None else -1
        HP, EP, NTP = self.HP, self.EP, self.NTP
        shapes = [('emb', (V, EP)), ('w_ih', (2, 4 * HP, EP)), ('w_hh', (2, 4 * HP, HP)), ('b_ih', (2, 4 * HP)),
                  ('b_hh', (2, 4 * HP)), ('w_out', (NTP, 2 * HP)), ('b_out', (NTP,))]
        self._seg, o = {}, 0
        for k, sh in shapes:
            self._seg[k] = (o, sh)
            o += int(np.prod(sh))
        self.numel = o
        f = dict(device=dev, dtype=torch.float32)
        self.w, self.g, self.m, self.v = (torch.zeros(o, **f) for _ in range(4))
        self.ctr = torch.zeros(4, device=dev, dtype=torch.int32)       # [0]: steps taken (Adam t, dropout)
        self.loss_sum = torch.zeros(4, **f)                              # [0]: sum of batch-mean losses
        self.whhT = torch.empty((2, HP, 4 * HP), **f)
        self.bsum = torch.empty(8 * HP, **f)
        self.lr, self.p, self.seed = float(lr), float(dropout), int(seed) & ((1 << 63) - 1)
        self.betas, self.eps = betas, eps
        self.device = dev
        self._graphs, self._inbuf, self._pool = {}, {}, None
        self._pinned, self._events, self._flip = [None, None], [None, None], 0
        self.load_module(net)

    # ------------------------------------------------------------------------ parameters
    def seg(self, t: torch.Tensor, k: str) -> torch.Tensor:
        o, sh = self._seg[k]
        return t[o:o + int(np.prod(sh))].view(sh)

    @torch.no_grad()
    def load_module(self, net):
        E, H, HP, NT = self.E, self.H, self.HP, self.NT
        self.w.zero_()
        self.seg(self.w, 'emb')[:, :E] = net.emb.weight.float()
        for d, suf in enumerate(('', '_reverse')):
            l = net.lstm
            self.seg(self.w, 'w_ih').view(2, 4, HP, self.EP)[d, :, :H, :E] = \
                getattr(l, 'weight_ih_l0' + suf).float().view(4, H, E)
            self.seg(self.w, 'w_hh').view(2, 4, HP, HP)[d, :, :H, :H] = \
                getattr(l, 'weight_hh_l0' + suf).float().view(4, H, H)
            self.seg(self.w, 'b_ih').view(2, 4, HP)[d, :, :H] = getattr(l, 'bias_ih_l0' + suf).float().view(4, H)
            self.seg(self.w, 'b_hh').view(2, 4, HP)[d, :, :H] = getattr(l, 'bias_hh_l0' + suf).float().view(4, H)
        self.seg(self.w, 'w_out').view(self.NTP, 2, HP)[:NT, :, :H] = net.out.weight.float().view(NT, 2, H)
        self.seg(self.w, 'b_out')[:NT] = net.out.bias.float()

    def _unpad(self, t: torch.Tensor) -> dict:
        """Module-shaped views (copies) of an arena (weights or gradients)."""
        E, H, HP, NT = self.E, self.H, self.HP, self.NT
        out = {'emb.weight': self.seg(t, 'emb')[:, :E].clone(),
               'out.weight': self.seg(t, 'w_out').view(self.NTP, 2, HP)[:NT, :, :H].reshape(NT, 2 * H).clone(),
               'out.bias': self.seg(t, 'b_out')[:NT].clone()}
        for d, suf in enumerate(('', '_reverse')):
            out['lstm.weight_ih_l0' + suf] = self.seg(t, 'w_ih').view(2, 4, HP, self.EP)[d, :, :H, :E].reshape(4 * H, E)
            out['lstm.weight_hh_l0' + suf] = self.seg(t, 'w_hh').view(2, 4, HP, HP)[d, :, :H, :H].reshape(4 * H, H)
            out['lstm.bias_ih_l0' + suf] = self.seg(t, 'b_ih').view(2, 4, HP)[d, :, :H].reshape(4 * H)
            out['lstm.bias_hh_l0' + suf] = self.seg(t, 'b_hh').view(2, 4, HP)[d, :, :H].reshape(4 * H)
        return {k: v.clone() for k, v in out.items()}

    @torch.no_grad()
    def store_module(self, net):
        sd = net.state_dict()
        for k, v in self._unpad(self.w).items():
            sd[k].copy_(v.to(sd[k].dtype))

    def grads(self) -> dict:
        return self._unpad(self.g)

    def state(self) -> dict:
        return {'w': self.w.cpu(), 'm': self.m.cpu(), 'v': self.v.cpu(), 'ctr': self.ctr.cpu(), 'seed': self.seed}

    def load_state(self, st: dict):
        for k in ('w', 'm', 'v', 'ctr'):
            getattr(self, k).copy_(st[k])
        self.seed = int(st['seed'])

    # ------------------------------------------------------------------------ the step
    def _body(self, ib: torch.Tensor, L: int, B: int, update: bool = True):
        n, HP, EP, NTP = L * B, self.HP, self.EP, self.NTP
        dev, f, s = self.device, torch.float32, _s()
        ids, labels, perm = ib[0:n], ib[n:2 * n], ib[2 * n:3 * n]
        uniq, starts, nruns = ib[3 * n:4 * n], ib[4 * n:5 * n + 1], ib[5 * n + 1:5 * n + 2]
        inv = ib[5 * n + 2:5 * n + 3]
        W, G = self.w, self.g
        if update:   # t of Adam's bias corrections and the dropout stream's step
            _lib.call("rk_add_int", _p(self.ctr), 1, s)
        x = torch.empty((n, EP), device=dev, dtype=f)
        mask = torch.empty((n, EP), device=dev, dtype=f) if self.p > 0 else None
        _lib.call("rk_tag_embed_fwd", _p(ids), _p(self.seg(W, 'emb')), _p(x), _p(mask), n, EP, self.V, self.p,
                  self.seed, _DROP_STREAM, _p(self.ctr), s)
        self.last_mask = mask   # (tests: the dropout multipliers of the latest eager step, time-major rows)
        _lib.call("rk_tag_add", _p(self.seg(W, 'b_ih')), _p(self.seg(W, 'b_hh')), _p(self.bsum), 8 * HP, s)
        w_ih = self.seg(W, 'w_ih').view(8 * HP, EP)
        gin = S.linear(x, w_ih, self.bsum)
        hout = torch.empty((L, B, 2, HP), device=dev, dtype=f)
        gsave = torch.empty((L, B, 2, 4 * HP), device=dev, dtype=f)
        csave = torch.empty((L, B, 2, HP), device=dev, dtype=f)
        _lib.call("rk_lstm_fwd32", _p(gin), _p(self.seg(W, 'w_hh')), L, B, HP, _p(hout), _p(gsave), _p(csave), s)
        h2 = hout.view(n, 2 * HP)
        w_out = self.seg(W, 'w_out')
        logits = S.linear(h2, w_out, self.seg(W, 'b_out'))
        dlog = torch.empty((n, NTP), device=dev, dtype=f)
        _lib.call("rk_softmax_xent_f32s", _p(logits), NTP, _p(labels), n, self.NT, IGNORE, _p(inv), _p(dlog), NTP,
                  _p(self.loss_sum), s)
        S.linear_dw(dlog, h2, out=self.seg(G, 'w_out'))
        S.colsum(dlog, self.seg(G, 'b_out'))
        dh = S.linear_dx(dlog, w_out)
        _lib.call("rk_tag_transpose", _p(self.seg(W, 'w_hh')), _p(self.whhT), 2, 4 * HP, HP, s)
        dg = torch.empty((L, B, 2, 4 * HP), device=dev, dtype=f)
        _lib.call("rk_lstm_bwd32", _p(self.whhT), L, B, HP, _p(dh), _p(gsave), _p(csave), _p(dg), s)
        dg2 = dg.view(n, 8 * HP)
        S.linear_dw(dg2, x, out=self.seg(G, 'w_ih').view(8 * HP, EP))
        g_hh = self.seg(G, 'w_hh')
        if L > 1:   # h_{t-1} of the forward direction, h_{t+1} of the reverse one (zero initial state)
            S.linear_dw(dg2[B:, :4 * HP], h2[:-B, :HP], out=g_hh[0])
            S.linear_dw(dg2[:-B, 4 * HP:], h2[B:, HP:], out=g_hh[1])
        else:
            _lib.call("rk_zero32", _p(g_hh), g_hh.numel(), s)
        S.colsum(dg2, self.seg(G, 'b_ih').view(-1))
        _lib.call("rk_tag_add", _p(self.seg(G, 'b_ih')), None, _p(self.seg(G, 'b_hh')), 8 * HP, s)
        gx = S.linear_dx(dg2, w_ih)
        g_emb = self.seg(G, 'emb')
        _lib.call("rk_zero32", _p(g_emb), g_emb.numel(), s)
        _lib.call("rk_tag_embed_bwd", _p(perm), _p(uniq), _p(starts), _p(nruns), _p(gx), _p(mask), _p(g_emb), n, EP,
                  self.V, s)
        if update:
            b1, b2 = self.betas
            _lib.call("rk_adam_step", _p(self.w), None, _p(self.g), _p(self.m), _p(self.v), self.numel, self.lr, b1, b2,
                      1.0 - b1, 1.0 - b2, self.eps, 0.0, 0, 1.0, 1.0, 1.0, None, _p(self.ctr), s)

    def _upload(self, words: np.ndarray, key) -> torch.Tensor:
        """Async copy of a packed batch into the shape's device input buffer (pinned, double-buffered)."""
        k = self._flip
        self._flip ^= 1
        buf = self._pinned[k]
        if buf is None or buf.numel() < words.size:
            if self._events[k] is not None:
                self._events[k].synchronize()
            buf = self._pinned[k] = torch.empty(max(words.size, 1 << 16), dtype=torch.int32, pin_memory=True)
        elif self._events[k] is not None:
            self._events[k].synchronize()     # the copy that last read this buffer has run
        buf[:words.size].numpy()[:] = words
        dst = self._inbuf.get(key)
        if dst is None:
            dst = self._inbuf[key] = torch.empty(words.size, dtype=torch.int32, device=self.device)
        dst.copy_(buf[:words.size], non_blocking=True)
        ev = self._events[k] = torch.cuda.Event()
        ev.record()
        return dst

    def step(self, x_bl: np.ndarray, y_bl: np.ndarray, update: bool = True, graph: bool = True):
        """One training step on a batch-first [B, L] batch (ids int, labels IGNORE-padded)."""
        B, L = x_bl.shape
        key = (L, B)
        ib = self._upload(pack_batch(x_bl, y_bl, self.padding_idx, self.V), key)
        g = self._graphs.get(key) if graph and update else None
        if g is not None:
            g.replay()
            return
        self._body(ib, L, B, update)
        if graph and update:
            # the eager run tuned this shape's GEMMs; capture for the next batches of this shape
            with graphs.LOCK:
                torch.cuda.current_stream().synchronize()
                if self._pool is None:
                    self._pool = torch.cuda.graph_pool_handle()
                cg = torch.cuda.CUDAGraph()
                with graphs.capture(cg, pool=self._pool):
                    self._body(ib, L, B, True)   # recorded, not run: the eager run above was this step
                self._graphs[key] = cg

    def take_loss(self) -> float:
        """Sum of the batch-mean losses since the last call (one host sync)."""
        v = float(self.loss_sum[0].item())
        _lib.call("rk_zero32", _p(self.loss_sum), 4, _s())
        return v

    # ------------------------------------------------------------------------ inference
    @torch.no_grad()
    def logits(self, x_bl: np.ndarray) -> torch.Tensor:
        """[B, L, tags] logits (eval: no dropout), eager on the same kernels."""
        B, L = x_bl.shape
        n, HP, EP, dev, s = B * L, self.HP, self.EP, self.device, _s()
        ids = torch.from_numpy(np.ascontiguousarray(x_bl.T, dtype=np.int32).reshape(-1)).to(dev)
        x = torch.empty((n, EP), device=dev, dtype=torch.float32)
        _lib.call("rk_tag_embed_fwd", _p(ids), _p(self.seg(self.w, 'emb')), _p(x), None, n, EP, self.V, 0.0, 0, 0,
                  None, s)
        _lib.call("rk_tag_add", _p(self.seg(self.w, 'b_ih')), _p(self.seg(self.w, 'b_hh')), _p(self.bsum), 8 * HP, s)
        gin = S.linear(x, self.seg(self.w, 'w_ih').view(8 * HP, EP), self.bsum)
        hout = torch.empty((L, B, 2, HP), device=dev, dtype=torch.float32)
        gsave = torch.empty((L, B, 2, 4 * HP), device=dev, dtype=torch.float32)
        csave = torch.empty((L, B, 2, HP), device=dev, dtype=torch.float32)
        _lib.call("rk_lstm_fwd32", _p(gin), _p(self.seg(self.w, 'w_hh')), L, B, HP, _p(hout), _p(gsave), _p(csave), s)
        lg = S.linear(hout.view(n, 2 * HP), self.seg(self.w, 'w_out'), self.seg(self.w, 'b_out'))
        return lg.view(L, B, self.NTP)[:, :, :self.NT].transpose(0, 1)

    def close(self):
        with graphs.quiesced():
            self._graphs.clear()
