"""Where does the fused F(4x4) forward kernel's time go?  Times rk_wino4_conv from several builds of
winograd4.hip compiled with experiment macros (WEXP_NOMFMA / NOLOAD / NOSTORE: skip the MFMAs, the
global loads or the transform + LDS writes) on the VGG-small 32x32 / 16x16 shapes.
usage: python scripts/dev/wino_breakdown.py scripts/dev/exp_so/w4_*.so > out.jsonl"""
import ctypes as C
import json
import os
import sys

import torch

vp, i32 = C.c_void_p, C.c_int


def t(fn, reps=30):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


shapes = [(256, 32, 64, 64), (256, 16, 64, 128), (256, 16, 128, 128)]
bufs = {}
for (N, H, Ci, Co) in shapes:
    x = torch.randn(N, H, H, Ci, device='cuda')
    u = torch.randn(36, Co, Ci, device='cuda') * 0.05
    y = torch.empty(N, H, H, Co, device='cuda')
    st = torch.zeros(64, 2, Co, dtype=torch.float64, device='cuda')
    bufs[(N, H, Ci, Co)] = (x, u, y, st)

for path in sys.argv[1:]:
    lib = C.CDLL(os.path.abspath(path))
    f = lib.rk_wino4_conv
    f.argtypes = [vp, vp, vp, vp, vp, i32, vp, i32, i32, i32, i32, i32, i32, i32, vp]
    for key, (x, u, y, st) in bufs.items():
        N, H, Ci, Co = key
        for var in (0, 1):
            def run():
                rc = f(x.data_ptr(), u.data_ptr(), y.data_ptr(), None, st.data_ptr(), 63, None, N, H, H, Ci, Co, 4,
                       var, C.c_void_p(torch.cuda.current_stream().cuda_stream))
                assert rc == 0, rc
            us = t(run)
            print(json.dumps(dict(build=os.path.basename(path), N=N, H=H, Ci=Ci, Co=Co, variant=var,
                                  us=round(us, 1))), flush=True)
