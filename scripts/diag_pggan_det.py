"""Where does PG-GAN run-to-run nondeterminism enter?  Two identically-seeded models, stage by stage of
one D step (G forward, D forward, GP gradient, D backward) and one G step; prints max |diff| per stage.
usage: python scripts/diag_pggan_det.py"""
import json
import sys

sys.path.insert(0, '.')
import torch  # noqa: E402

from rafiki_amd.engine.flat import FlatAdam  # noqa: E402
from rafiki_amd.models.pg_gan import PgGan, TrialRng  # noqa: E402
from rafiki_amd.ops import _lib  # noqa: E402

_lib.lib()
DEV = torch.device('cuda', 0)


def build():
    m = PgGan(D_repeats=1, minibatch_base=16, fmap_base=1024, fmap_max=128, seed=3)
    m.device = DEV
    m._build([1, 16, 16], 0)
    return m


def stages(m, lod=2.0, mb=64):
    nets = m.nets
    out = {}
    rng = TrialRng(DEV, 11)
    level = torch.randint(0, 256, (256, 1, 4, 4), dtype=torch.uint8, generator=torch.Generator().manual_seed(1)).to(DEV)
    PG, PD = nets.src_G(), nets.src_D()
    nets.set_requires_grad(nets.g_params, False)
    nets.set_requires_grad(nets.d_params, True)
    nets.D.grad.zero_()
    idx = m._shard(rng.randint(level.shape[0], mb, TrialRng.D_IDX)).to(level.device)
    reals = m._reals(level, idx, lod - int(lod))
    labels = torch.zeros((mb, 0), device=DEV)
    with torch.no_grad():
        fakes = nets.generator(PG, m._latents(mb, rng, TrialRng.D_LAT), labels, lod)
    out['G_fwd'] = fakes.detach().clone()
    rf_s, _ = nets.discriminator(PD, torch.cat([reals, fakes.to(reals.dtype)], 0), lod, segs=2)
    out['D_fwd'] = rf_s.detach().clone()
    alpha = m._shard(rng.rand((mb, 1, 1, 1), TrialRng.D_ALPHA))
    mixed = (reals.float() + (fakes.float() - reals.float()) * alpha).to(reals.dtype).detach().requires_grad_(True)
    mixed_s, _ = nets.discriminator(PD, mixed, lod)
    (grads,) = torch.autograd.grad(mixed_s.sum(), mixed, create_graph=True)
    out['GP_grad'] = grads.detach().clone()
    norms = grads.float().square().sum((1, 2, 3)).sqrt()
    loss = (rf_s[mb:] - rf_s[:mb]) + (norms - 1.0).square() * 10.0 + rf_s[:mb].square() * 0.001
    loss.mean().backward(retain_graph=True)
    out['D_grad'] = nets.D.grad.clone()
    nets.D.grad.zero_()
    (mixed_s.sum()).backward(retain_graph=True)
    out['D_grad_plain'] = nets.D.grad.clone()
    nets.D.grad.zero_()
    (norms.sum()).backward()
    out['D_grad_gp_only'] = nets.D.grad.clone()
    # G step
    nets.set_requires_grad(nets.d_params, False)
    nets.set_requires_grad(nets.g_params, True)
    nets.G.grad.zero_()
    fk = nets.generator(PG, m._latents(mb, rng, TrialRng.G_LAT), labels, lod)
    fs, _ = nets.discriminator(PD, fk, lod)
    (-fs).mean().backward()
    out['G_grad'] = nets.G.grad.clone()
    torch.cuda.synchronize()
    return out


warm = build()
stages(warm)            # autotunes every shape once
a, b = build(), build()
assert torch.equal(a.nets.G.master, b.nets.G.master) and torch.equal(a.nets.D.master, b.nets.D.master)
sa, sb = stages(a), stages(b)
sa2 = stages(a)         # the same model again
res = {}
for k in sa:
    d1 = (sa[k] - sb[k]).abs().max().item()
    d2 = (sa[k] - sa2[k]).abs().max().item()
    res[k] = {'max_abs_diff_models': d1, 'max_abs_diff_rerun': d2, 'scale': sa[k].abs().max().item()}
print(json.dumps(res, indent=1))
