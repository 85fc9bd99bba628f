"""Native BiLSTM tagger step (engine/tagger.py, csrc/kernels/tagger.hip) vs fp64 torch references.

Reference model: examples/models/pos_tagging/PyBiLstm.py:249-268 (Embedding(padding_idx=0) -> Dropout ->
BiLSTM -> Linear, cross-entropy over the non-padding tokens, Adam).  Shapes are deliberately unaligned
(E = 37, H = 51, 45 tags, odd batch sizes): the engine's padded arena keeps them on the in-tree kernels.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


class Net(torch.nn.Module):
    def __init__(self, V, E, H, NT, p=0.0):
        super().__init__()
        self.emb = torch.nn.Embedding(V, E, padding_idx=0)
        self.drop = torch.nn.Dropout(p)
        self.lstm = torch.nn.LSTM(E, H, batch_first=True, bidirectional=True)
        self.out = torch.nn.Linear(2 * H, NT)


def _batch(rng, B, L, V, NT):
    lens = rng.integers(1, L + 1, B)
    lens[0] = L
    x = np.zeros((B, L), np.int64)
    y = np.full((B, L), -100, np.int64)
    for b, n in enumerate(lens):
        x[b, :n] = rng.integers(1, V, n)
        x[b, min(n, 2) - 1] = 3                        # repeated ids: runs of several tokens
        y[b, :n] = rng.integers(0, NT, n)
    return x, y


def _ref_grads(net, x, y, mask=None):
    """fp64 CPU autograd of the reference computation; mask: [B, L, E] dropout multipliers."""
    ref = Net(net.emb.num_embeddings, net.emb.embedding_dim, net.lstm.hidden_size, net.out.out_features).double()
    ref.load_state_dict({k: v.detach().cpu().double() for k, v in net.state_dict().items()})
    e = ref.emb(torch.from_numpy(x))
    if mask is not None:
        e = e * mask
    h = ref.lstm(e)[0]
    logits = ref.out(h)
    loss = torch.nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]), torch.from_numpy(y).reshape(-1),
                                             ignore_index=-100)
    loss.backward()
    return {k: p.grad for k, p in ref.named_parameters()}, float(loss)


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("V,E,H,NT,B,L", [(50, 37, 51, 45, 5, 7), (120, 16, 64, 12, 33, 4), (40, 128, 128, 7, 3, 1),
                                          (64, 21, 100, 17, 9, 11)])
def test_tagger_grads_match_fp64(V, E, H, NT, B, L):
    from rafiki_amd.engine.tagger import TaggerEngine
    torch.manual_seed(0)
    net = Net(V, E, H, NT).to(DEV)
    eng = TaggerEngine(net, lr=0.01, dropout=0.0)
    rng = np.random.default_rng(1)
    x, y = _batch(rng, B, L, V, NT)
    eng.step(x, y, update=False, graph=False)
    torch.cuda.synchronize()
    g = eng.grads()
    ref, loss = _ref_grads(net, x, y)
    for k, r in ref.items():
        assert _rel(g[k].cpu(), r) < 1e-5, (k, _rel(g[k].cpu(), r))
    assert abs(eng.take_loss() - loss) < 1e-5 * max(1.0, abs(loss))
    # the padded arena's pad region got exactly zero gradient
    total = sum(int(v.numel()) for v in g.values())
    assert float(eng.g.abs().sum()) == pytest.approx(sum(float(v.abs().sum()) for v in g.values()), rel=1e-6)
    assert total <= eng.numel


def test_tagger_dropout_mask_and_grads():
    from rafiki_amd.engine.tagger import TaggerEngine
    torch.manual_seed(1)
    V, E, H, NT, B, L, p = 60, 37, 51, 45, 7, 9, 0.3
    net = Net(V, E, H, NT).to(DEV)
    eng = TaggerEngine(net, lr=0.01, dropout=p, seed=1234)
    rng = np.random.default_rng(2)
    x, y = _batch(rng, B, L, V, NT)
    eng.step(x, y, update=False, graph=False)
    torch.cuda.synchronize()
    m = eng.last_mask.cpu()[:, :E]                                   # [L*B, E] time-major
    vals = set(np.unique(m.numpy()).tolist())
    assert vals <= {0.0, np.float32(1.0 / (1.0 - p))}, vals
    keep = float((m > 0).float().mean())
    assert abs(keep - (1 - p)) < 0.05, keep
    mask = m.view(L, B, E).transpose(0, 1).double()
    ref, _ = _ref_grads(net, x, y, mask=mask)
    g = eng.grads()
    for k, r in ref.items():
        assert _rel(g[k].cpu(), r) < 1e-5, (k, _rel(g[k].cpu(), r))


def test_tagger_adam_update_matches_fp64():
    from rafiki_amd.engine.tagger import TaggerEngine
    torch.manual_seed(2)
    V, E, H, NT, B, L = 50, 37, 51, 45, 5, 6
    net = Net(V, E, H, NT).to(DEV)
    lr = 0.02
    eng = TaggerEngine(net, lr=lr, dropout=0.1, seed=7)
    rng = np.random.default_rng(3)
    b1, b2, eps = 0.9, 0.999, 1e-8
    for t in range(1, 4):
        w0, m0, v0 = eng.w.double().cpu(), eng.m.double().cpu(), eng.v.double().cpu()
        x, y = _batch(rng, B, L, V, NT)
        eng.step(x, y, graph=False)
        torch.cuda.synchronize()
        g = eng.g.double().cpu()
        m = b1 * m0 + (1 - b1) * g
        v = b2 * v0 + (1 - b2) * g * g
        w = w0 - lr * (m / (1 - b1 ** t)) / ((v / (1 - b2 ** t)).sqrt() + eps)
        assert int(eng.ctr[0]) == t
        assert _rel(eng.m.cpu(), m) < 1e-6 and _rel(eng.v.cpu(), v) < 1e-6
        assert float((eng.w.double().cpu() - w).abs().max()) < 1e-6


def test_tagger_graph_replay_matches_eager():
    """Captured-and-replayed steps (one graph per bucket shape) give bit-identical weights to eager
    steps over the same batches: same kernels, same device counter, same dropout stream."""
    from rafiki_amd.engine.tagger import TaggerEngine
    torch.manual_seed(3)
    V, E, H, NT = 70, 37, 51, 45
    net = Net(V, E, H, NT).to(DEV)
    a = TaggerEngine(net, lr=0.01, dropout=0.2, seed=99)
    b = TaggerEngine(net, lr=0.01, dropout=0.2, seed=99)
    rng = np.random.default_rng(4)
    shapes = [(5, 7), (3, 4), (5, 7), (5, 7), (3, 4), (8, 2), (5, 7)]
    for B, L in shapes:
        x, y = _batch(rng, B, L, V, NT)
        a.step(x, y, graph=True)
        b.step(x, y, graph=False)
    torch.cuda.synchronize()
    assert len(a._graphs) == 3
    assert torch.equal(a.w, b.w) and torch.equal(a.m, b.m) and torch.equal(a.v, b.v)
    la, lb = a.take_loss(), b.take_loss()   # summed with float atomics: order-dependent in the last bits
    assert abs(la - lb) <= 1e-5 * max(1.0, abs(lb)), (la, lb)
    a.close()


def test_pybilstm_native_trains_unaligned_knobs():
    """The PyBiLstm model on the native engine at knob values that are not multiples of 4."""
    from rafiki_amd.models.pos_tagging import PyBiLstm
    m = PyBiLstm(epochs=3, word_embed_dims=37, word_rnn_hidden_size=51, word_dropout=0.01, learning_rate=0.05,
                 batch_size=32)
    m.train("synthetic://corpus?n=400&seed=0")
    assert m._engine is not None
    acc = m.evaluate("synthetic://corpus?n=100&seed=1")
    assert acc > 0.5, acc
    out = m.predict([["a", "b", "c"]])
    assert len(out) == 1 and len(out[0]) == 3
