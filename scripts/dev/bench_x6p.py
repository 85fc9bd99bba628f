"""Pre-split X6 GEMM (x6p.hip) on the 36-group GEMMs of the VGG-small pre-transformed F(4x4) layers
(batch 256): microseconds and fp32-equivalent TFLOP/s of every tile / ring depth, against the X6 bf16
peak (2.5 PFLOP/s / 6 products = 417 TFLOP/s).  usage: python scripts/dev/bench_x6p.py [out.jsonl]
X6P_CFGS="tile,nst,splits;..." restricts the configs; X6P_SHARED=1 gives every group the SAME A and B (group
strides 0: the operands stay L2-resident — separates L2/HBM supply from the CU-side intake); RAFIKI_X6P_DBG=1|2
(tiles 0 / 3): no DMA in the K loop | no MFMAs."""
import json
import os
import sys

sys.path.insert(0, '.')
import torch  # noqa: E402

from rafiki_amd.ops import _lib, f32 as S  # noqa: E402

_lib.lib()
PEAK = 2.5e15 / 6


def t(fn, reps=20):
    if os.environ.get('X6P_EAGER') == '1':   # plain launches (profiler counter passes)
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return 1.0
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    s.record()
    g.replay()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


# (name, M, N, K): conv fwd/dgrad Y'[q] = V[q] U[q]^T (M = tiles, N = out channels, K = in channels) and
# weight gradients dU[q] = M^T[q] V^T[q]^T (M = Cout, N = Cin, K = tiles)
SHAPES = [('c5f', 1024, 256, 256), ('c6f', 256, 512, 256), ('c7f', 256, 512, 512), ('c4d', 1024, 128, 256),
          ('c6d', 256, 256, 512), ('c5w', 256, 256, 1024), ('c7w', 512, 512, 256)]
res = []
SHARED = os.environ.get('X6P_SHARED') == '1'


def phases(tile, M, N, sp):
    """Per-block phase stamps of the last launch (RAFIKI_X6P_DBG & 4): median shader-clock cycles of the
    prologue (start -> first K-tile landed), the K loop and the epilogue, the clock (MHz) and the block
    start spread (how many rounds of blocks the grid ran in)."""
    import numpy as np
    bm, bn = S.XP_TILES[tile & 15]
    nb = -(-M // bm) * -(-N // bn) * 36 * sp
    h = np.zeros(nb * 8, dtype=np.uint64)
    torch.cuda.synchronize()
    _lib.call("rk_x6p_stamps", h.ctypes.data, nb * 8)
    h = h.reshape(nb, 8).astype(np.float64)
    pro, loop, epi = h[:, 1] - h[:, 0], h[:, 2] - h[:, 1], h[:, 3] - h[:, 2]
    mhz = (h[:, 3] - h[:, 0]) / np.maximum(1.0, h[:, 5] - h[:, 4]) * 100.0
    life = h[:, 3] - h[:, 0]
    span = h[:, 3].max() - h[:, 0].min()
    return {'blocks': nb, 'prologue': float(np.median(pro)), 'loop': float(np.median(loop)),
            'epilogue': float(np.median(epi)), 'life': float(np.median(life)), 'mhz': float(np.median(mhz)),
            'span_cycles': float(span), 'concurrency': float(life.sum() / max(1.0, span))}


def gemm(a, b, out, M, N, K, tile, nst, sp):
    if not SHARED:
        return S.x6p_gemm(a, b, out, M, N, K, groups=36, tile=tile, nst=nst, splits=sp)
    _lib.call("rk_x6p_gemm", tile, nst, a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, K, K, N, M * K, N * K,
              0, 0, M * N, 36, 0, sp, 36 * M * N, a.numel() * 2, b.numel() * 2, torch.cuda.current_stream().cuda_stream)


if os.environ.get('X6P_SHAPES'):
    SHAPES = [x for x in SHAPES if x[0] in os.environ['X6P_SHAPES'].split(',')]
for name, M, N, K in SHAPES:
    a = torch.randn(1 if SHARED else 36, 3, M, K, device='cuda').to(torch.bfloat16)
    b = torch.randn(1 if SHARED else 36, 3, N, K, device='cuda').to(torch.bfloat16)
    out = torch.empty(4, 36, M, N, device='cuda')
    fl = 2.0 * 36 * M * N * K
    r = dict(name=name, M=M, N=N, K=K, shared=SHARED, dbg=os.environ.get('RAFIKI_X6P_DBG', '0'))
    times = {}
    cfgs = [(t + kt, n, sp) for (t, n, sp) in S._XP_CFGS for kt in (0, 16) if not (kt and K % 64)]
    if os.environ.get('X6P_CFGS'):   # e.g. "3,2,1;16,3,1" (timing-diagnostic runs: RAFIKI_X6P_DBG)
        cfgs = [tuple(int(v) for v in c.split(',')) for c in os.environ['X6P_CFGS'].split(';')]
    for (tile, nst, sp) in cfgs:
        sp = S.x6p_splits(K, sp)
        try:
            times[(tile, nst, sp)] = t(lambda: gemm(a, b, out[:sp], M, N, K, tile, nst, sp))
            if int(os.environ.get('RAFIKI_X6P_DBG', '0')) & 4 and tile & 15 in (0, 3):
                r.setdefault('phases', {})['{},{},{}'.format(tile, nst, sp)] = phases(tile, M, N, sp)
        except Exception:  # noqa: BLE001
            times[(tile, nst, sp)] = float('inf')
    best = min(times, key=times.get)
    r['best'] = list(best)
    r['us'] = round(times[best], 2)
    r['tflops'] = round(fl / times[best] / 1e6, 1)
    r['pct_x6_peak'] = round(100 * fl / (times[best] * 1e-6) / PEAK, 1)
    r['all'] = {'{},{},{}'.format(*k): round(v, 1) for k, v in times.items()}
    print(json.dumps(r), flush=True)
    res.append(r)
if len(sys.argv) > 1:
    with open(sys.argv[1], 'w') as f:
        for r in res:
            f.write(json.dumps(r) + '\n')
