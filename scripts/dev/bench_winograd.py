"""Fused Winograd F(2x2,3x3) fp32 conv vs the direct implicit-GEMM conv on the VGG-small layer shapes
(batch 256, BN statistics epilogue).  usage: python scripts/dev/bench_winograd.py"""
import sys, time, json
sys.path.insert(0, '.')
import torch
from rafiki_amd.ops import f32 as S, _lib
_lib.lib()
res = []
for (N, H, C, K) in [(256, 32, 64, 64), (256, 16, 64, 128), (256, 16, 128, 128), (256, 8, 128, 256), (256, 8, 256, 256), (256, 4, 256, 512), (256, 4, 512, 512)]:
    x = torch.randn(N, H, H, C, device='cuda')
    w = torch.randn(K, 9 * C, device='cuda') * 0.05
    u = torch.empty(16, K, C, device='cuda'); ut = torch.empty(16, C, K, device='cuda')
    S.wino_weights(w, u, ut)
    acc = torch.zeros((S.bn_slots(K), 2, K), dtype=torch.float64, device='cuda')
    def t(fn, reps=20):
        fn(); torch.cuda.synchronize()
        s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps): fn()
        e.record(); e.synchronize()
        return s.elapsed_time(e) / reps * 1e3
    tw0 = t(lambda: S.wino_conv(x, u, stats=acc, variant=0))
    tw1 = t(lambda: S.wino_conv(x, u, stats=acc, variant=1))
    tw = min(tw0, tw1)
    td = t(lambda: S.conv_fwd(x, w.view(K, 3, 3, C), stats_acc=acc))
    tt = t(lambda: S.wino_weights(w, u, ut))
    dy = torch.randn(N, H, H, K, device='cuda')
    dw = torch.empty(K, 9 * C, device='cuda')
    tww = {c[2]: t(lambda: S.wino_wgrad(dy, x, dw, splits=c[2])) for c in S._wino_wgrad_cands(N, H, H, K, C)}
    s_best = min(tww, key=tww.get) if tww else None
    twd = t(lambda: S.conv_wgrad(dy, x, out=dw))
    fl = 2.0 * N * H * H * K * 9 * C
    res.append(dict(N=N, H=H, C=C, K=K, wino4_us=round(tw0, 1), wino8_us=round(tw1, 1), direct_us=round(td, 1), wt_us=round(tt, 1),
                    speedup=round(td / tw, 2), wino_eff_tflops=round(fl / tw / 1e6, 1),
                    wgrad_wino_us=round(tww[s_best], 1) if tww else None, wgrad_splits=s_best,
                    wgrad_direct_us=round(twd, 1)))
    print(json.dumps(res[-1]), flush=True)
