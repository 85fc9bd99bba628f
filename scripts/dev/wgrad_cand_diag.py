"""Error of every conv_wgrad autotune candidate vs fp64 on given shapes (diagnostic)."""
import json
import sys
import torch
sys.path.insert(0, '.')
from rafiki_amd.ops import f32 as S

res = []


def each(key, cands, run, protect=()):
    return cands


for (N, H, Cin, Cout) in [(16, 48, 4, 16), (16, 48, 8, 16), (16, 32, 4, 16), (16, 24, 4, 16), (64, 48, 4, 64)]:
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, H, H, Cin, generator=g).cuda()
    dy = torch.randn(N, H, H, Cout, generator=g).cuda()
    ref = torch.nn.grad.conv2d_weight(x.double().cpu().permute(0, 3, 1, 2), (Cout, Cin, 3, 3),
                                      dy.double().cpu().permute(0, 3, 1, 2), padding=1)   # [co][ci][3][3]
    ref = ref.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin)
    orig = S._pick
    cands = {}

    def grab(key, c, run, protect=()):
        cands['list'] = list(c)
        cands['run'] = run
        return c[0]
    S._pick = grab
    out = torch.zeros(Cout, 9 * Cin, device='cuda')
    S.conv_wgrad(dy, x, out=out)
    S._pick = orig
    for c in cands['list']:
        out.zero_()
        try:
            cands['run'](c)
            torch.cuda.synchronize()
            e = ((out.double().cpu() - ref).norm() / ref.norm()).item()
        except Exception as ex:
            e = repr(ex)[:80]
        print(json.dumps(dict(N=N, H=H, Cin=Cin, Cout=Cout, cfg=list(c), err=e)), flush=True)
