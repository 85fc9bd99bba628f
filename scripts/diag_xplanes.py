"""Diagnostic: the X6 weight planes written by WinoWeights' multi-layer refresh vs the single-layer
transform, for every layer of the full-width fp32 engine."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('RAFIKI_XCONV', '1')
import torch  # noqa: E402

from rafiki_amd.engine.convnet import ConvNetEngine  # noqa: E402
from rafiki_amd.ops import f32 as S  # noqa: E402

eng = ConvNetEngine(num_classes=10, in_channels=3, image_size=32, cfg=(64, 64, 'M', 128, 128, 'M', 256, 256, 'M', 512,
                                                                       512, 'M'), fc_dims=(512,), device='cuda',
                    seed=3, lr=0.05, dtype='fp32')
ww = eng._wino_train()
print('live', sorted(k for k in ww.live if k[0] in ('x', 'xt')))
ww.refresh()
torch.cuda.synchronize()
for l, b in enumerate(eng.blocks):
    w = eng.flat.w(b[0] + '.w')
    for kind, dg in (('x', False), ('xt', True)):
        if not ww.has(kind, l):
            continue
        got = ww._view(kind, l).clone()
        ref = S.xconv_planes(w, dgrad=dg)
        torch.cuda.synchronize()
        print(l, kind, tuple(got.shape), 'equal' if torch.equal(got, ref) else 'DIFF max {:.3e}'.format(
            (got.float() - ref.float()).abs().max().item()))
# the other sets must be untouched by the X6 refresh: compare with a fresh transform
for l, b in enumerate(eng.blocks):
    w = eng.flat.w(b[0] + '.w').reshape(b[2], -1)
    for kind, fn in (('u4', S.wino4_u), ('ut4', S.wino4_ut), ('u2', S.wino_u), ('ut2', S.wino_ut)):
        if ww.has(kind, l):
            got = ww._view(kind, l)
            ref = fn(w)
            print(l, kind, 'equal' if torch.allclose(got, ref, rtol=0, atol=0) else 'DIFF {:.3e}'.format(
                (got - ref).abs().max().item()))
