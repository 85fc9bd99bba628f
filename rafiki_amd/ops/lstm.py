"""Bidirectional LSTM on the persistent gfx950 recurrence kernels (csrc/kernels/lstm.hip).

Reference: examples/models/pos_tagging/PyBiLstm.py:249-268 (``nn.LSTM(Ew, h, batch_first=True,
bidirectional=True)`` over a padded batch, zero initial state).  Split of the work:

* the input projection ``x @ W_ih^T + b_ih + b_hh`` of every timestep and both directions is one
  GEMM on the in-tree fp32 kernels (``ops.f32.linear``: sgemm.hip, f32 / X6 loops, autotuned, bias in
  the epilogue), as are the backward's input gradient (``linear_dx``), the two weight gradients
  (``linear_dw``, W_hh's per direction over strided views) and the bias gradient (``colsum``) — they
  have no time dependence;
* the word embedding (PyBiLstm.py:249) is ``embedding``: an in-tree gather kernel forward and a
  deterministic sort + segmented-sum scatter backward (csrc/kernels/embed.hip);
* the sequential part (T steps of ``h @ W_hh^T`` + the cell) is ONE kernel launch per direction
  pair, forward and backward: ``rk_lstm_fwd32`` / ``rk_lstm_bwd32`` (exact fp32 on
  v_mfma_f32_16x16x4_f32, the reference's precision, default) or ``rk_lstm_fwd`` / ``rk_lstm_bwd``
  (bf16 W_hh and h operands, fp32 cell state and accumulation; opt-in with ``dtype='bf16'``).

Hidden sizes are zero-padded per gate block to HP in {64, 128}; padded units stay exactly zero,
so the result equals the unpadded LSTM.  On CPU (or hidden > 128) ``bilstm`` runs torch's LSTM.
"""
from __future__ import annotations

import torch

from . import _lib
from . import f32 as S
from .functional import _p, _s


def _native_dense(*dims) -> bool:
    """The in-tree fp32 GEMMs take 16-B (4-float) rows: every non-batch extent a multiple of 4."""
    return all(d % 4 == 0 for d in dims)


class EmbeddingFn(torch.autograd.Function):
    """out = W[ids] (rk_embedding_fwd); dW by a stable sort of the token ids and an in-order segmented sum
    per id (rk_embedding_bwd: bit-reproducible, no float atomics); padding_idx's row gets no gradient."""

    @staticmethod
    def forward(ctx, ids, w, padding_idx):
        ids = ids.contiguous().to(torch.int64)
        n, (V, E) = ids.numel(), w.shape
        out = torch.empty(ids.shape + (E,), device=w.device, dtype=torch.float32)
        _lib.call("rk_embedding_fwd", _p(ids), _p(w.contiguous()), _p(out), n, E, V, _s())
        ctx.save_for_backward(ids)
        ctx.dims = (V, E, -1 if padding_idx is None else int(padding_idx))
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gy):
        (ids,) = ctx.saved_tensors
        V, E, pad = ctx.dims
        n = ids.numel()
        gw = torch.empty((V, E), device=gy.device, dtype=torch.float32)
        nbytes = int(_lib.lib().rk_embedding_bwd_ws(n))
        ws = torch.empty(nbytes, device=gy.device, dtype=torch.uint8)
        _lib.call("rk_embedding_bwd", _p(ids), _p(gy.contiguous().float()), _p(gw), n, V, E, pad, _p(ws), nbytes, _s())
        return None, gw, None


def embedding(ids, emb: torch.nn.Embedding):
    """``emb(ids)`` on the gfx950 kernels (fp32 weights, E % 4 == 0); torch's own elsewhere."""
    w = emb.weight
    if ids.device.type != 'cuda' or w.dtype != torch.float32 or w.shape[1] % 4 or emb.max_norm is not None:
        return emb(ids)
    return EmbeddingFn.apply(ids, w, emb.padding_idx)


def _hp(H: int) -> int:
    return 64 if H <= 64 else 128


def _pad_gate_rows(w: torch.Tensor, H: int, HP: int) -> torch.Tensor:
    """[2, 4H, ...] -> [2, 4HP, ...] with each gate block zero-padded from H to HP rows."""
    rest = w.shape[2:]
    out = w.new_zeros((2, 4, HP) + tuple(rest))
    out[:, :, :H] = w.reshape((2, 4, H) + tuple(rest))
    return out.reshape((2, 4 * HP) + tuple(rest))


class BiLstmFn(torch.autograd.Function):
    """x [T, B, E] fp32, w_ih [2, 4H, E], w_hh [2, 4H, H], b [2, 4H] (b_ih + b_hh) -> [T, B, 2H].
    ``dtype`` picks the recurrence kernels: 'fp32' (default) or 'bf16'."""

    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b, dtype='fp32'):
        T, B, E = x.shape
        H = w_hh.shape[-1]
        HP = _hp(H)
        w_ih_p = _pad_gate_rows(w_ih.detach().float(), H, HP)                          # [2, 4HP, E]
        w_hh_p = torch.zeros((2, 4 * HP, HP), device=x.device, dtype=torch.float32)
        w_hh_p[:, :, :H] = _pad_gate_rows(w_hh.detach().float(), H, HP)
        f32 = dtype != 'bf16'
        # fp32: W_hh as is for the forward, W_hh^T [2, HP, 4HP] for the BPTT (float4 along k)
        w_rec = w_hh_p.contiguous() if f32 else w_hh_p.to(torch.bfloat16).contiguous()
        b_p = _pad_gate_rows(b.detach().float(), H, HP)                                  # [2, 4HP]
        x2 = x.detach().float().reshape(T * B, E).contiguous()
        if _native_dense(E):
            gin = S.linear(x2, w_ih_p.reshape(2 * 4 * HP, E), b_p.reshape(-1).contiguous())
        else:
            gin = torch.addmm(b_p.reshape(1, -1), x2, w_ih_p.reshape(2 * 4 * HP, E).t()).contiguous()
        hout = torch.empty((T, B, 2, HP), device=x.device, dtype=torch.float32)
        gsave = torch.empty((T, B, 2, 4 * HP), device=x.device, dtype=torch.float32)
        csave = torch.empty((T, B, 2, HP), device=x.device, dtype=torch.float32)
        _lib.call("rk_lstm_fwd32" if f32 else "rk_lstm_fwd", _p(gin), _p(w_rec), T, B, HP, _p(hout), _p(gsave),
                  _p(csave), _s())
        if f32:
            w_rec = w_hh_p.transpose(1, 2).contiguous()
        ctx.save_for_backward(x2, w_ih_p, w_rec, hout, gsave, csave)
        ctx.dims = (T, B, E, H, HP)
        ctx.f32 = f32
        return hout[..., :H].reshape(T, B, 2 * H)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gy):
        x2, w_ih_p, w_rec, hout, gsave, csave = ctx.saved_tensors
        T, B, E, H, HP = ctx.dims
        dh = torch.zeros((T, B, 2, HP), device=gy.device, dtype=torch.float32)
        dh[..., :H] = gy.reshape(T, B, 2, H)
        dg = torch.empty((T, B, 2, 4 * HP), device=gy.device, dtype=torch.float32)
        _lib.call("rk_lstm_bwd32" if ctx.f32 else "rk_lstm_bwd", _p(w_rec), T, B, HP, _p(dh), _p(gsave), _p(csave),
                  _p(dg), _s())
        dg2 = dg.reshape(T * B, 2 * 4 * HP)
        native = _native_dense(E)
        gx = gw_ih = gw_hh = gb = None
        if ctx.needs_input_grad[0]:
            w2 = w_ih_p.reshape(2 * 4 * HP, E)
            gx = (S.linear_dx(dg2, w2) if native else dg2 @ w2).reshape(T, B, E)
        if ctx.needs_input_grad[1]:
            gw = S.linear_dw(dg2, x2) if native else \
                torch.einsum('ndg,ne->dge', dg2.reshape(T * B, 2, 4 * HP), x2)            # [2, 4HP, E]
            gw_ih = gw.reshape(2, 4, HP, E)[:, :, :H].reshape(2, 4 * H, E)
        if ctx.needs_input_grad[2]:
            # h_{t-1} of the forward direction / h_{t+1} of the reverse one (zero initial state)
            hp = torch.zeros_like(hout)
            hp[1:, :, 0] = hout[:-1, :, 0]
            hp[:-1, :, 1] = hout[1:, :, 1]
            gw = torch.empty((2, 4 * HP, HP), device=gy.device, dtype=torch.float32)
            for d in range(2):   # per direction over strided row views: [TB, 4HP]^T [TB, HP]
                S.linear_dw(dg.view(T * B, 2, 4 * HP)[:, d], hp.view(T * B, 2, HP)[:, d], out=gw[d])
            gw_hh = gw.reshape(2, 4, HP, HP)[:, :, :H, :H].reshape(2, 4 * H, H)
        if ctx.needs_input_grad[3]:
            gsum = torch.empty(2 * 4 * HP, device=gy.device, dtype=torch.float32)
            S.colsum(dg2, gsum)
            gb = gsum.reshape(2, 4, HP)[:, :, :H].reshape(2, 4 * H)
        return gx, gw_ih, gw_hh, gb, None


def bilstm(x, lstm: torch.nn.LSTM, dtype='fp32'):
    """Run a 1-layer bidirectional ``nn.LSTM`` (batch_first) on the gfx950 kernels; returns
    [B, T, 2H] like ``lstm(x)[0]``.  CPU tensors and hidden > 128 use torch's own LSTM."""
    H = lstm.hidden_size
    if x.device.type != 'cuda' or H > 128 or lstm.num_layers != 1 or not lstm.bidirectional:
        return lstm(x)[0]
    w_ih = torch.stack([lstm.weight_ih_l0, lstm.weight_ih_l0_reverse])
    w_hh = torch.stack([lstm.weight_hh_l0, lstm.weight_hh_l0_reverse])
    b = torch.stack([lstm.bias_ih_l0 + lstm.bias_hh_l0, lstm.bias_ih_l0_reverse + lstm.bias_hh_l0_reverse])
    y = BiLstmFn.apply(x.transpose(0, 1).contiguous(), w_ih, w_hh, b, dtype)
    return y.transpose(0, 1)
