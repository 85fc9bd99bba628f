"""VGG-style static-graph engine on the GPU, opt-in bf16 compute path (dtype='bf16'), vs the PyTorch
fp32 reference of the same network.  The default fp32 path is covered by tests/test_f32_gpu.py."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _engine(**kw):
    from rafiki_amd.engine.convnet import ConvNetEngine
    args = dict(num_classes=10, in_channels=3, image_size=16, cfg=(16, 'M', 32, 32, 'M'), fc_dims=(32,),
                device='cuda', seed=3, lr=0.05, dtype='bf16')
    args.update(kw)
    return ConvNetEngine(**args)


def _batch(B, hw=16, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.zeros(B, hw, hw, 8)
    x[..., :3] = torch.randn(B, hw, hw, 3, generator=g)
    y = torch.randint(0, 10, (B,), generator=g, dtype=torch.int32)
    return x.bfloat16().cuda(), y.cuda()


def test_grads_match_reference():
    eng = _engine()
    x, y = _batch(64)
    eng.forward_backward(x, y)
    torch.cuda.synchronize()
    fl = eng.flat
    params = {n: fl.w(n).detach().clone().requires_grad_(True) for n in fl.names()}
    # tight oracle: fp32 reference with bf16 rounding (straight-through) where the engine stores bf16
    loss, _ = eng.reference_loss(x, y, params, training=True, emulate_bf16=True)
    grads = torch.autograd.grad(loss, [params[n] for n in fl.names()])
    assert abs(eng.loss_sum.item() / 64 - loss.item()) < 1e-2 * max(1.0, loss.item())
    for n, g in zip(fl.names(), grads):
        got = fl.g(n)
        fro = ((got - g).norm() / g.norm().clamp_min(1e-12)).item()
        cos = torch.nn.functional.cosine_similarity(got.flatten(), g.flatten(), 0).item()
        # residual = independent bf16 rounding of dy feeding the (cancelling) sum_p dy*x reduction
        print('bf16-grad-vs-emulated', n, round(fro, 4), round(cos, 5))
        assert fro < 0.12 and cos > 0.99, (n, fro, cos)
    # loose oracle: plain fp32 reference (bf16 storage shifts pool routing: direction must agree)
    loss32, _ = eng.reference_loss(x, y, params, training=True)
    g32 = torch.autograd.grad(loss32, [params[n] for n in fl.names()])
    for n, g in zip(fl.names(), g32):
        cos = torch.nn.functional.cosine_similarity(fl.g(n).flatten(), g.flatten(), 0).item()
        assert cos > 0.97, (n, cos)


def test_bf16_bn_backward_is_exact_given_its_inputs(monkeypatch):
    """Localises the ~5% residual of the bf16 engine vs the bf16-emulating oracle (test above).
    Every BN(+ReLU, +2x2 max-pool) backward of the engine — including the sums fused into the dgrad
    epilogues — reproduces an fp64 autograd BatchNorm backward of ITS OWN inputs (bf16 y and incoming
    gradient) to < 1% (measured 0.2%).  The oracle's inputs differ from the engine's by ~1% (another
    bf16 rounding realisation of the same network: measured 1.3% on the last block's incoming
    gradient), and the BN backward's cancelling projection dz = k1*(g - mean g - xhat*mean(g*xhat))
    amplifies that ~4x (measured 5.4% on its output) — so the end-to-end
    gate above stays loose by construction while the kernels are pinned tightly here."""
    import torch.nn.functional as TF
    from rafiki_amd.ops import functional as F
    eng = _engine()
    x, y = _batch(64)
    cap = []
    orig = F.bn_bwd_acc

    def bb(d, yy, coeffs, gamma, acc, **kw):
        out = orig(d, yy, coeffs, gamma, acc, **kw)
        cap.append((d.clone(), yy.clone(), out.clone(), kw.get('pool', False)))
        return out
    monkeypatch.setattr(F, 'bn_bwd_acc', bb)
    eng.forward_backward(x, y)
    torch.cuda.synchronize()
    assert len(cap) == len(eng.blocks)
    for k, bi in enumerate(range(len(eng.blocks) - 1, -1, -1)):
        d, yb, dz, pool = cap[k]
        name = eng.blocks[bi][0]
        y64 = yb.double().cpu().permute(0, 3, 1, 2).requires_grad_(True)
        h = torch.relu(TF.batch_norm(y64, None, None, eng.flat.w(name + '.gamma').double().cpu(),
                                     eng.flat.w(name + '.beta').double().cpu(), training=True, eps=eng.bn_eps))
        if pool:
            h = TF.max_pool2d(h, 2)
        (ref,) = torch.autograd.grad(h, y64, d.double().cpu().permute(0, 3, 1, 2))
        got = dz.double().cpu().permute(0, 3, 1, 2)
        err = ((got - ref).norm() / ref.norm()).item()
        print('bn backward vs fp64 of its inputs', name, round(err, 5))
        assert err < 1e-2, (name, err)


def test_graph_replay_matches_eager():
    e1, e2 = _engine(), _engine()
    e2.capture(32)
    for i in range(3):
        x, y = _batch(32, seed=i)
        e1.train_step(x, y)
        e2.step_graph(x, y)
    torch.cuda.synchronize()
    assert torch.equal(e1.flat.master, e2.flat.master)
    assert torch.allclose(e1.running, e2.running)


@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_scheduled_graph_matches_eager_and_advances_counter(opt):
    """capture_scheduled: one prologue kernel gathers rows sched[ctr] and zeroes the BN slot tables; the
    step counter advances in the SGD kernel (sgd) or in the prologue once every block has read it
    (adam); replays must track an eager loop over the same rows."""
    e1, e2 = _engine(optimizer=opt, lr=0.01 if opt == 'adam' else 0.05), _engine(optimizer=opt,
                                                                               lr=0.01 if opt == 'adam' else 0.05)
    data, labels = _batch(96, seed=7)
    steps, B = 4, 32
    idx = torch.randint(0, 96, (steps, B), device='cuda', generator=torch.Generator('cuda').manual_seed(1))
    e2.capture_scheduled(data, labels, steps, B)
    e2.set_schedule(idx)
    for i in range(steps):
        e1.train_step(data[idx[i]].contiguous(), labels[idx[i]].contiguous())
        e2.replay()
    torch.cuda.synchronize()
    assert int(e2._ctr.item()) == steps and int(e2._done.item()) == 0
    assert torch.allclose(e1.flat.master, e2.flat.master, rtol=1e-5, atol=1e-6)
    assert torch.allclose(e1.running, e2.running, rtol=1e-4, atol=1e-6)
    assert abs(e1.loss_sum.item() - e2.loss_sum.item()) < 1e-3 * max(1.0, abs(e1.loss_sum.item()))


def test_scheduled_graph_with_a_one_step_schedule():
    """A dataset smaller than two batches gives a one-row schedule; the capture's warm-up steps (and any
    replay past the schedule) must wrap around it, never read past the schedule or the dataset."""
    e1, e2 = _engine(lr=0.05), _engine(lr=0.05)
    data, labels = _batch(40, seed=3)
    B = 32
    e2.capture_scheduled(data, labels, 1, B)
    g = torch.Generator('cuda').manual_seed(2)
    for ep in range(3):
        idx = torch.randperm(40, device='cuda', generator=g)[:B].view(1, B)
        e2.set_schedule(idx)
        e1.train_step(data[idx[0]].contiguous(), labels[idx[0]].contiguous())
        e2.replay()
    torch.cuda.synchronize()
    assert int(e2._ctr.item()) == 1
    assert torch.allclose(e1.flat.master, e2.flat.master, rtol=1e-5, atol=1e-6)


def test_training_reduces_loss_and_eval():
    eng = _engine(lr=0.05)
    x, y = _batch(128, seed=5)
    eng.capture(128)
    losses = []
    for _ in range(30):
        eng.reset_metrics()
        eng.step_graph(x, y)
        losses.append(eng.loss_sum.item() / 128)
    assert losses[-1] < 0.5 * losses[0], losses
    probs = eng.forward_eval(x)
    assert torch.allclose(probs.sum(1), torch.ones(128, device='cuda'), atol=1e-4)
    _, ref_logits = eng.reference_loss(x, None, training=False)
    ref = torch.softmax(ref_logits, 1)
    assert (probs - ref).abs().max().item() < 5e-2


def test_grads_match_reference_non_pow2_vgg16_layout():
    """48x48 input with VGG16-style pooling to 3x3 -> 1x1 (non-power-of-two gather + odd pool)."""
    eng = _engine(image_size=48, cfg=(16, 'M', 32, 'M', 32, 'M', 64, 'M', 64, 'M'), fc_dims=(64,))
    x, y = _batch(32, hw=48, seed=7)
    eng.forward_backward(x, y)
    torch.cuda.synchronize()
    fl = eng.flat
    params = {n: fl.w(n).detach().clone().requires_grad_(True) for n in fl.names()}
    loss, _ = eng.reference_loss(x, y, params, training=True, emulate_bf16=True)
    grads = torch.autograd.grad(loss, [params[n] for n in fl.names()])
    assert abs(eng.loss_sum.item() / 32 - loss.item()) < 1e-2 * max(1.0, loss.item())
    for n, g in zip(fl.names(), grads):
        got = fl.g(n)
        fro = ((got - g).norm() / g.norm().clamp_min(1e-12)).item()
        cos = torch.nn.functional.cosine_similarity(got.flatten(), g.flatten(), 0).item()
        # 5 BN stages down to 1x1 at batch 32 amplify the bf16 dy rounding; the same net at 32x32 (the
        # power-of-two path) measures fro 0.18 / cos 0.983 on conv0
        print('bf16-grad48-vs-emulated', n, round(fro, 4), round(cos, 5))
        assert fro < 0.2 and cos > 0.98, (n, fro, cos)


@pytest.mark.parametrize("bn", [False, True])
def test_vgg16_model_trains(bn):
    """Vgg16 trains end to end: the default Keras-VGG16 network (conv + bias + ReLU, no BatchNorm, fp32)
    at Adam 1e-4 — plain 16-layer VGG from scratch needs the smaller step Keras users give it — and the
    batch_norm knob's conv + BN + ReLU blocks at 1e-3."""
    import numpy as np
    from rafiki_amd.models.vgg16 import Vgg16
    m = Vgg16(epochs=1, learning_rate=1e-3 if bn else 1e-4, batch_size=32, batch_norm=bn)
    m._knobs['epochs'] = 6 if bn else 10
    m.train('synthetic://image?n=512&size=28&channels=1&classes=4&seed=0')
    acc = m.evaluate('synthetic://image?n=256&size=28&channels=1&classes=4&seed=1')
    assert acc > 0.5, acc
    p = m.predict([np.zeros((28, 28), np.uint8).tolist()])
    assert len(p) == 1 and abs(sum(p[0]) - 1) < 1e-3


def test_graphed_eval_matches_eager_for_large_batches():
    """Batches above the largest bucket are chunked; every chunk must survive the next replay."""
    eng = _engine()
    x, y = _batch(1100, seed=9)
    eng.train_step(x[:64], y[:64])
    eng.prepare_eval()
    a = eng.forward_eval_graphed(x).clone()
    b = eng.forward_eval(x)
    assert a.shape == b.shape and torch.allclose(a, b, atol=1e-5)


def test_mlp_model_learns_on_gpu():
    from rafiki_amd.model.model import load_model_class
    from rafiki_amd.models import model_file
    clazz = load_model_class(open(model_file('FeedForward'), 'rb').read(), 'FeedForward')
    m = clazz(epochs=3, hidden_layer_count=2, hidden_layer_units=64, learning_rate=0.001, batch_size=128,
              image_size=28, dtype='bf16')
    m.train('synthetic://image?n=3000&size=28&channels=1&classes=10&seed=0')
    assert m.evaluate('synthetic://image?n=1500&size=28&channels=1&classes=10&seed=1') > 0.9
