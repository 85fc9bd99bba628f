"""gfx950 numerics for the PG-GAN / VGG16 kernel extensions and the twice-differentiable Functions.

* fused nearest-upscale + conv3x3 (kind 6) vs F.conv2d(upsample(x));
* non-power-of-two channel counts (the 512+1 -> 520 minibatch-stddev conv) and spatial extents
  (VGG16 at 48x48: 48/24/12/6/3) for conv fwd / dgrad / wgrad;
* WGAN-GP double backward through the GPU Functions vs the CPU fp32 PyTorch oracle.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def fn():
    from rafiki_amd.ops import _lib, functional
    _lib.lib()
    return functional


def _nchw(x):
    return x.permute(0, 3, 1, 2)


@pytest.mark.parametrize("N,h,Cin,Cout", [(4, 4, 512, 512), (2, 8, 64, 128), (8, 2, 32, 64), (3, 16, 16, 8)])
def test_conv_upscale_fused(fn, N, h, Cin, Cout):
    torch.manual_seed(0)
    x = torch.randn(N, h, h, Cin, device=DEV).bfloat16()
    w = (torch.randn(Cout, 3, 3, Cin, device=DEV) / (3 * Cin ** 0.5)).bfloat16()
    b = torch.randn(Cout, device=DEV)
    y = fn.conv_up(x, w, bias=b, act=fn.ACT_LRELU, slope=0.2)
    up = F.interpolate(_nchw(x.float()), scale_factor=2, mode="nearest")
    ref = F.leaky_relu(F.conv2d(up, w.float().permute(0, 3, 1, 2), b, padding=1), 0.2).permute(0, 2, 3, 1)
    assert y.shape == (N, 2 * h, 2 * h, Cout)
    assert rel_err(y, ref) < 1e-2


SHAPES = [(4, 4, 4, 520, 512), (2, 48, 48, 64, 64), (4, 6, 6, 128, 128), (8, 3, 3, 512, 256), (3, 12, 12, 24, 40),
          (2, 24, 24, 136, 64)]


@pytest.mark.parametrize("N,H,W,Cin,Cout", SHAPES)
def test_conv_nonpow2_fwd_dgrad_wgrad(fn, N, H, W, Cin, Cout):
    torch.manual_seed(1)
    x = torch.randn(N, H, W, Cin, device=DEV).bfloat16()
    w = (torch.randn(Cout, 3, 3, Cin, device=DEV) / (3 * Cin ** 0.5)).bfloat16()
    wr = w.float().permute(0, 3, 1, 2)
    y = fn.conv_fwd(x, w)
    ref = F.conv2d(_nchw(x.float()), wr, padding=1).permute(0, 2, 3, 1)
    assert rel_err(y, ref) < 1e-2
    dy = torch.randn(N, H, W, Cout, device=DEV).bfloat16()
    if Cout & (Cout - 1) == 0:  # dgrad's tap-major weight rows need a power-of-two Cout
        dx = fn.conv_dgrad(dy, w)
        rdx = torch.nn.grad.conv2d_input((N, Cin, H, W), wr, _nchw(dy.float()), padding=1).permute(0, 2, 3, 1)
        assert rel_err(dx, rdx) < 1e-2
    dw = fn.conv_wgrad(dy, x)
    rdw = torch.nn.grad.conv2d_weight(_nchw(x.float()), (Cout, Cin, 3, 3), _nchw(dy.float()),
                                      padding=1).permute(0, 2, 3, 1).reshape(Cout, -1)
    assert rel_err(dw, rdw) < 5e-3


def _twin_nets(res=8, fmap_base=256, fmap_max=64):
    from rafiki_amd.models.pg_gan import PgNetworks
    g = PgNetworks(num_channels=1, resolution=res, fmap_base=fmap_base, fmap_max=fmap_max, device=DEV, seed=3)
    c = PgNetworks(num_channels=1, resolution=res, fmap_base=fmap_base, fmap_max=fmap_max, device='cpu', seed=3)
    return g, c


def _gp_loss(nets, x, lod):
    P = nets.src_D()
    xi = x.clone().requires_grad_(True)
    s, _ = nets.discriminator(P, xi, lod)
    (gr,) = torch.autograd.grad(s.sum(), xi, create_graph=True)
    norms = gr.float().square().sum((1, 2, 3)).sqrt()
    return s.float(), gr.float(), ((norms - 1) ** 2 * 10 + s.float().square() * 1e-3).mean()


@pytest.mark.parametrize("lod", [0.0, 0.5])
def test_wgan_gp_double_backward_matches_fp32(lod):
    """Scores, input gradients and GP weight-gradients of the bf16 gfx950 path track the fp32 oracle."""
    gnet, cnet = _twin_nets()
    torch.manual_seed(0)
    x = torch.randn(8, 8, 8, gnet.cpad)
    x[..., 1:] = 0
    s_g, gr_g, loss_g = _gp_loss(gnet, x.to(DEV).bfloat16(), lod)
    s_c, gr_c, loss_c = _gp_loss(cnet, x.bfloat16().float(), lod)
    assert cos(s_g.cpu(), s_c) > 0.99
    assert cos(gr_g.cpu(), gr_c) > 0.98
    gnet.D.grad.zero_()
    cnet.D.grad.zero_()
    loss_g.backward()
    loss_c.backward()
    torch.cuda.synchronize()
    for name in ('8x8/Conv0/weight', '8x8/Conv1_down/weight', '4x4/Conv/weight', '4x4/Dense0/weight',
                 'FromRGB_lod0/weight'):
        a, b = gnet.D.g(name).cpu(), cnet.D.g(name)
        assert cos(a, b) > 0.97, (name, cos(a, b))


def test_generator_upconv_path_matches_fp32():
    gnet, cnet = _twin_nets(res=16)
    torch.manual_seed(1)
    lat = torch.randn(8, gnet.latent_size)
    lab = torch.zeros(8, 0)
    img_g = gnet.generator(gnet.src_G(), lat.to(DEV), lab.to(DEV), 0.0)
    img_c = cnet.generator(cnet.src_G(), lat, lab, 0.0)
    assert img_g.shape == (8, 16, 16, gnet.cpad)
    assert cos(img_g.float().cpu(), img_c) > 0.99
    img_g.float().square().mean().backward()
    img_c.square().mean().backward()
    for name in ('16x16/Conv0_up/weight', '8x8/Conv1/weight', '4x4/Dense/weight'):
        a, b = gnet.G.g(name).cpu(), cnet.G.g(name)
        assert cos(a, b) > 0.97, (name, cos(a, b))


def test_pg_gan_trains_on_gpu(tmp_path, monkeypatch):
    monkeypatch.setenv("RAFIKI_OUTPUT_DIR", str(tmp_path))
    from rafiki_amd.models.pg_gan import PgGan
    m = PgGan(D_repeats=2, minibatch_base=8, G_lrate=1e-3, D_lrate=1e-3, lod_initial_resolution=4, total_kimg=2.0,
              lod_training_kimg=0.6, lod_transition_kimg=0.6, fmap_base=1024, fmap_max=256, eval_images=512)
    m.train("synthetic://image?n=1024&size=16&channels=1&classes=4&seed=0")
    assert all(math.isfinite(v) for v in m.stats.values()), m.stats
    s = m.evaluate("synthetic://image?n=512&size=16&channels=1&classes=4&seed=1")
    assert 1.0 <= s <= 4.0 + 1e-6
    paths = m.predict([2, 2, 1])
    assert len(paths) == 1
