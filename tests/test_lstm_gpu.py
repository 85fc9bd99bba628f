"""gfx950 persistent BiLSTM kernels (rafiki_amd.ops.lstm) vs torch's fp32 nn.LSTM on the CPU."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-30)).item()


def rel_err(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("B,T,E,H", [(16, 7, 32, 64), (37, 12, 48, 128), (5, 3, 16, 20), (130, 9, 64, 100)])
def test_bilstm_matches_fp32_lstm(B, T, E, H, dtype):
    from rafiki_amd.ops import _lib
    from rafiki_amd.ops.lstm import bilstm
    _lib.lib()
    torch.manual_seed(0)
    ref = torch.nn.LSTM(E, H, batch_first=True, bidirectional=True)
    gpu = torch.nn.LSTM(E, H, batch_first=True, bidirectional=True).to(DEV)
    gpu.load_state_dict(ref.state_dict())
    x = torch.randn(B, T, E)
    gy = torch.randn(B, T, 2 * H)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)[0]
    (yr * gy).sum().backward()
    xg = x.to(DEV).requires_grad_(True)
    yg = bilstm(xg, gpu, dtype=dtype)
    (yg * gy.to(DEV)).sum().backward()
    assert yg.shape == yr.shape
    if dtype == "fp32":   # exact-precision recurrence: fp32 rounding-level agreement with torch's CPU LSTM
        assert rel_err(yg.cpu(), yr) < 1e-4
        assert rel_err(xg.grad.cpu(), xr.grad) < 1e-4
        for name, p in ref.named_parameters():
            g = dict(gpu.named_parameters())[name].grad
            assert g is not None, name
            assert rel_err(g.cpu(), p.grad) < 2e-4, name
        return
    assert rel_err(yg.cpu(), yr) < 2e-2 and cos(yg.cpu(), yr) > 0.9999
    assert cos(xg.grad.cpu(), xr.grad) > 0.999
    for name, p in ref.named_parameters():
        g = dict(gpu.named_parameters())[name].grad
        assert g is not None, name
        assert cos(g.cpu(), p.grad) > 0.998, name


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_pybilstm_trains_on_gpu(dtype):
    from rafiki_amd.models.pos_tagging import PyBiLstm
    tr = "synthetic://corpus?n=400&seed=0"
    te = "synthetic://corpus?n=100&seed=1"
    m = PyBiLstm(epochs=3, word_embed_dims=32, word_rnn_hidden_size=48, word_dropout=0.01, learning_rate=0.05,
                 batch_size=32, dtype=dtype)
    m.train(tr)
    acc = m.evaluate(te)
    assert acc > 0.5, acc
    out = m.predict([["a", "b", "c"]])
    assert len(out) == 1 and len(out[0]) == 3
