"""CPU test of WinoWeights' live-set bookkeeping (rafiki_amd/ops/f32.py): which Winograd weight sets a
step refreshes, the on-demand transform of a set outside the live group, and that narrowing never
happens while a hipGraph capture is open.  The kernel launcher is replaced by a recorder, so this
runs without a GPU; the GPU test test_winograd4_gpu.py checks the transformed values themselves."""
import torch

from rafiki_amd.ops import f32 as S


class Recorder:
    def __init__(self):
        self.calls = []

    def __call__(self, name, *args):
        self.calls.append((name, args))
        return 0

    def names(self):
        return [c[0] for c in self.calls]


def _setup(monkeypatch, capturing=False):
    rec = Recorder()
    monkeypatch.setattr(S._lib, 'call', rec)
    monkeypatch.setattr(S, '_s', lambda: None)
    monkeypatch.setattr(S, '_p', lambda t: None if t is None else t.data_ptr())   # host tensors are fine here
    monkeypatch.setattr(torch.cuda, 'is_current_stream_capturing', lambda: capturing)
    shapes = [(64, 32), (16, 64), (40, 24)]
    arena = torch.zeros(sum(co * 9 * ci for co, ci in shapes) + 3)
    ws, off = [], 3
    for co, ci in shapes:
        ws.append(arena[off:off + co * 9 * ci].view(co, 9 * ci))
        off += co * 9 * ci
    ww = S.WinoWeights(arena, ws, hw=[8, 6, 4], f4=True)
    return rec, ww


def _tables(ww):
    """{family: {layer: (u_offset, ut_offset)}} of the tables refresh() launches with."""
    out = {}
    layer_of = {so: l for l, (so, _, _) in enumerate(ww._layers)}
    for fam, desc, meta, nb in ww._prepare(ww.live):
        m = meta.view(-1, 5)
        rows = sorted({int(x) for x in desc.view(-1, 4)[:, 0]})   # meta rows the blocks point at
        assert rows == list(range(m.shape[0])) and nb == desc.view(-1, 4).shape[0]
        out[fam] = {layer_of[int(m[r, 0])]: (int(m[r, 1]), int(m[r, 2])) for r in rows}
    return out


def test_sets_per_layer_follow_map_size(monkeypatch):
    _, ww = _setup(monkeypatch)
    # X6 planes of the pre-split PT path where its GEMM takes the shape (K = channels % 32, both >= 32)
    assert ww.has('u4p', 0) and ww.has('ut4p', 0) and not ww.has('u4p', 2) and not ww.has('ut4p', 2)
    assert ww.u4p(0).shape == (36, 3, 64, 32) and ww.u4p(0).dtype == torch.bfloat16
    assert ww.has('u2', 1) and ww.has('ut2', 1) and not ww.has('u4', 1)   # 6x6 map: no F(4x4) set
    assert ww.has('u4', 0) and ww.has('ut4', 2)
    assert ww.u4(1) is None and ww.u4(0).shape == (36, 64, 32) and ww.ut(2).shape == (16, 24, 40)
    # blocked sets of the UB fused kernels: rows padded to 32, flat
    assert ww.has('u4b', 0) and ww.has('ut4b', 2) and not ww.has('u4b', 1)
    assert ww._view('u4b', 2).shape == (36 * 64 * 24,) and ww._view('ut4b', 0).shape == (36 * 32 * 64,)


def test_refresh_narrows_to_the_sets_a_step_used(monkeypatch):
    rec, ww = _setup(monkeypatch)
    ww.refresh()
    assert rec.names() == ['rk_wino_weights_all']
    ww.end_step()                      # nothing read: keep everything
    assert len(ww.live) == 16
    ww.refresh()
    ww.lazy('u4', 0)()
    ww.lazy('ut2', 2)()
    ww.end_step()
    assert ww.live == frozenset({('u4', 0), ('ut2', 2)})
    t = _tables(ww)
    assert set(t) == {'2', '4'}
    # the plane family's meta rows carry offsets in bf16 elements (twice the float offset)
    ww.live = frozenset({('u4p', 0), ('ut4p', 0)})
    tp = _tables(ww)['p']
    assert tp == {0: (2 * ww._sets[('u4p', 0)][0], 2 * ww._sets[('ut4p', 0)][0])}
    ww.live = frozenset({('u4', 0), ('ut2', 2)})
    assert t['2'] == {2: (-1, ww._sets[('ut2', 2)][0])}          # gradient set only
    assert t['4'] == {0: (ww._sets[('u4', 0)][0], -1)}           # forward set only
    rec.calls.clear()
    ww.refresh()
    assert rec.names() == ['rk_wino_weights_all']
    # a set outside the live group is transformed on demand, once per step
    ww.lazy('u2', 1)()
    ww.lazy('u2', 1)()
    ww.lazy('ut4b', 2)()
    assert rec.names()[1:] == ['rk_wino_weights', 'rk_wino4b_weights']
    _, bargs = rec.calls[2]
    assert bargs[1] is None and bargs[2] is not None and bargs[3:5] == (40, 24)   # gradient set only
    _, args = rec.calls[1]
    assert args[1] is not None and args[2] is None                 # forward set, no gradient set


def test_no_narrowing_inside_capture(monkeypatch):
    rec, ww = _setup(monkeypatch, capturing=True)
    ww.refresh()
    ww.lazy('u2', 0)()
    ww.end_step()
    assert len(ww.live) == 16                                      # tables cannot be rebuilt in a capture


def test_sconvwt_refresh_is_lazy(monkeypatch):
    rec = Recorder()
    monkeypatch.setattr(S._lib, 'call', rec)
    monkeypatch.setattr(S, '_s', lambda: None)
    monkeypatch.setattr(S, '_p', lambda t: None if t is None else t.data_ptr())
    arena = torch.zeros(16 * 9 * 8 + 8 * 9 * 16)
    wt = S.SConvWT(arena, [arena[:16 * 72].view(16, 3, 3, 8), arena[16 * 72:].view(8, 3, 3, 16)])
    wt.begin_step()
    assert rec.names() == []                                       # no tuned dgrad used it yet
    v = wt.lazy(1)()
    wt.lazy(0)()
    assert rec.names() == ['rk_swt'] and v.shape == (16, 9 * 8)
    wt.begin_step()
    wt.lazy(0)()
    assert rec.names() == ['rk_swt', 'rk_swt']


def test_single_launch_refresh_table_covers_every_family(monkeypatch):
    """One rk_wino_weights_all launch whose table is the per-family tables concatenated — meta rows
    renumbered, the family id in each block's 4th field."""
    rec, ww = _setup(monkeypatch)
    ww.refresh()
    assert rec.names() == ['rk_wino_weights_all']
    fams = ww._prepare(ww.live)
    desc, meta, nb = ww._tables[('all', ww.live)]
    d, m = desc.view(-1, 4), meta.view(-1, 5)
    assert nb == d.shape[0] == sum(f[3] for f in fams)
    assert m.shape[0] == sum(f[2].numel() // 5 for f in fams)
    fam_of = {'2': 0, '4': 1, 'p': 2, 'b': 3}
    row = 0
    base = 0
    for fam, fdesc, fmeta, fnb in fams:
        fd = fdesc.view(-1, 4)
        got = d[row:row + fnb]
        assert (got[:, 0] == fd[:, 0] + base).all() and (got[:, 1:3] == fd[:, 1:3]).all()
        assert (got[:, 3] == fam_of[fam]).all()
        assert torch.equal(m[base:base + fmeta.numel() // 5], fmeta.view(-1, 5))
        row += fnb
        base += fmeta.numel() // 5


# ---- per-step weight-transform cache and in-place gradient marks (ops/autograd.py), host-side logic
def test_cached_weight_transforms_logic():
    """_wt caches a marked leaf's derived forms by (kind, address, shape) only inside the context, never a
    non-leaf (gradient) tensor or an unmarked leaf, and the cache and marks are gone after the context."""
    import torch
    from rafiki_amd.ops import autograd as A
    w = torch.nn.Parameter(torch.randn(4, 9, 8))
    other = torch.nn.Parameter(torch.randn(4, 72))
    grad_like = torch.randn(4, 72) * 2
    calls = []

    def producer(tag):
        def f():
            calls.append(tag)
            return torch.full((1,), float(len(calls)))
        return f
    view = w.reshape(4, -1)
    assert A._wt('u4p', view, producer('a')) is not None
    A._wt('u4p', view, producer('a'))()
    assert calls == ['a']                                  # no context: the producer itself, uncached
    with A.cached_weight_transforms([w]):
        assert getattr(w, '_rk_wcache', False)
        r1 = A._wt('u4p', view, producer('b'))()
        r2 = A._wt('u4p', w.reshape(4, -1), producer('b'))()   # same leaf, same form: served from the cache
        r3 = A._wt('ut4p', view, producer('c'))()             # another form: its own entry
        A._wt('u4p', other.reshape(4, -1), producer('d'))()   # unmarked leaf: never cached
        A._wt('u4p', other.reshape(4, -1), producer('d'))()
        A._wt('u4p', grad_like, producer('e'))()             # a non-leaf tensor: never cached
        A._wt('u4p', grad_like, producer('e'))()
        assert r1 is r2 and r3 is not r1
    assert calls == ['a', 'b', 'c', 'd', 'd', 'e', 'e']
    assert not getattr(w, '_rk_wcache', False) and not A._WT['cache'] and A._WT['on'] == 0


def test_in_place_grad_marks_are_scoped():
    import torch
    from rafiki_amd.ops import autograd as A
    p = torch.nn.Parameter(torch.zeros(3))
    p.grad = torch.zeros(3)
    with A.accumulate_weight_grads_in_place([p]):
        assert p._rk_direct
        with torch.no_grad():
            # CPU tensors never take the native in-place path (the GPU kernels write the buffer)
            assert A._param_grad_buffer(p) is None
    assert not p._rk_direct
