"""TfVgg16 network parity (reference examples/models/image_classification/TfVgg16.py:115-130: Keras
``VGG16(include_top=True, weights=None, input_shape=(48, 48, 3), classes=k)``): the default ``Vgg16``
has no BatchNorm, its parameter count equals Keras VGG16's at 48x48x3, and the CPU reference path
of the conv3x3 + bias + ReLU engine equals an independent torch.nn twin."""
import torch
import torch.nn as nn

from rafiki_amd.engine.convnet import ConvNetEngine
from rafiki_amd.models.vgg16 import VGG16_CFG, Vgg16


def keras_vgg16_params(h, w, c, classes):
    """Keras VGG16 with the top: 13 conv3x3 (+bias), five 2x2 pools, Flatten, Dense 4096 x2, Dense(classes)."""
    n, cin, hw = 0, c, (h, w)
    for v in VGG16_CFG:
        if v == 'M':
            hw = (hw[0] // 2, hw[1] // 2)
            continue
        n += 9 * cin * v + v
        cin = v
    flat = hw[0] * hw[1] * cin
    return n + (flat * 4096 + 4096) + (4096 * 4096 + 4096) + (4096 * classes + classes)


def test_default_vgg16_is_the_keras_network():
    m = Vgg16(epochs=1, learning_rate=1e-3, batch_size=32)
    kw = m._engine_kwargs(10, 3, 48)
    assert kw['bn'] is False and kw['dtype'] == 'fp32'
    assert Vgg16.get_knob_config()['batch_norm'].value is False
    eng = ConvNetEngine(num_classes=10, in_channels=3, image_size=48, device='cpu', **kw)
    names = eng.flat.names()
    assert not any(n.endswith(('.gamma', '.beta')) for n in names)
    assert sum(1 for n in names if n.startswith('conv') and n.endswith('.b')) == 13
    assert eng.real_param_count() == keras_vgg16_params(48, 48, 3, 10) == 33638218
    # the opt-in BN variant: + gamma / beta per conv channel
    kw_bn = Vgg16(batch_norm=True)._engine_kwargs(10, 3, 48)
    assert kw_bn['bn'] is True
    eng_bn = ConvNetEngine(num_classes=10, in_channels=3, image_size=48, device='cpu', **kw_bn)
    assert eng_bn.real_param_count() == 33638218 + sum(v for v in VGG16_CFG if v != 'M')


def test_no_bn_reference_path_matches_torch_nn_twin():
    torch.manual_seed(0)
    cfg = (8, 'M', 16, 16, 'M')
    eng = ConvNetEngine(num_classes=5, in_channels=3, image_size=16, cfg=cfg, fc_dims=(32,), device='cpu', bn=False)
    for b in eng.blocks:   # non-zero biases
        eng.flat.w(b[0] + '.b').copy_(torch.randn(b[2]) * 0.1)
    layers, cin = [], 3
    for v in cfg:
        if v == 'M':
            layers.append(nn.MaxPool2d(2))
            continue
        layers += [nn.Conv2d(cin, v, 3, padding=1), nn.ReLU()]
        cin = v
    twin = nn.Sequential(*layers, nn.Flatten(), nn.Linear(4 * 4 * 16, 32), nn.ReLU(), nn.Linear(32, 5)).double()
    convs = [l for l in twin if isinstance(l, nn.Conv2d)]
    fcs = [l for l in twin if isinstance(l, nn.Linear)]
    with torch.no_grad():
        for l, b in zip(convs, eng.blocks):
            w = eng.flat.w(b[0] + '.w')[..., :l.in_channels]   # [co][3][3][ci] (stem padded to cin_p)
            l.weight.copy_(w.permute(0, 3, 1, 2).double())
            l.bias.copy_(eng.flat.w(b[0] + '.b').double())
        # the engine flattens NHWC; the twin flattens NCHW: permute the first FC's input columns
        w0 = eng.flat.w('fc0.w')[:32].double().view(32, 4, 4, 16).permute(0, 3, 1, 2).reshape(32, -1)
        fcs[0].weight.copy_(w0)
        fcs[0].bias.copy_(eng.flat.w('fc0.b')[:32].double())
        fcs[1].weight.copy_(eng.flat.w('out.w')[:5, :32].double())
        fcs[1].bias.copy_(eng.flat.w('out.b')[:5].double())
    x = torch.randn(4, 16, 16, eng.cin_p, dtype=torch.float64)
    x[..., 3:] = 0
    _, logits = eng.reference_loss(x, None, params={n: eng.flat.w(n).double() for n in eng.flat.names()},
                                   training=False)
    ref = twin(x[..., :3].permute(0, 3, 1, 2))
    assert torch.allclose(logits, ref, rtol=1e-10, atol=1e-10)
