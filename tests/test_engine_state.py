"""CPU tests of engine state portability (the fp32 stem's padded input-channel count
depends on RAFIKI_WINOGRAD; params saved with one setting must load with the other)."""
import numpy as np
import torch

from rafiki_amd.engine.convnet import ConvNetEngine
from rafiki_amd.ops import f32 as S

CFG = (16, 'M', 16, 'M')


def _engine(monkeypatch, wino, seed=0):
    monkeypatch.setattr(S, 'WINO', wino)
    return ConvNetEngine(num_classes=10, in_channels=3, image_size=8, cfg=CFG, fc_dims=(16,), device='cpu',
                         seed=seed, dtype='fp32')


def test_stem_padding_differs(monkeypatch):
    assert _engine(monkeypatch, True).cin_p == 8
    assert _engine(monkeypatch, False).cin_p == 4


def test_save_wino_on_load_off_and_back(monkeypatch):
    a = _engine(monkeypatch, True, seed=1)
    sd = a.state_dict()
    b = _engine(monkeypatch, False, seed=2)
    b.load_state_dict(sd)
    wa, wb = sd['conv0.w'], b.state_dict()['conv0.w']
    assert wa.shape[-1] == 8 and wb.shape[-1] == 4
    np.testing.assert_array_equal(wa[..., :3], wb[..., :3])
    assert not wb[..., 3:].any()
    for k, v in sd.items():
        if k != 'conv0.w':
            np.testing.assert_array_equal(v, b.state_dict()[k])
    c = _engine(monkeypatch, True, seed=3)
    c.load_state_dict(b.state_dict())
    np.testing.assert_array_equal(c.state_dict()['conv0.w'], wa)


def test_nonzero_channels_are_not_dropped(monkeypatch):
    a = _engine(monkeypatch, True)
    sd = a.state_dict()
    sd['conv0.w'] = sd['conv0.w'].copy()
    sd['conv0.w'][..., 5] = 1.0
    b = _engine(monkeypatch, False)
    try:
        b.load_state_dict(sd)
    except ValueError as e:
        assert 'non-zero' in str(e)
    else:
        raise AssertionError('expected ValueError')
