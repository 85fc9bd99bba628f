"""Time every candidate config of a dense layer (split-K vs direct) — autotuner sanity check."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from rafiki_amd.ops import functional as F, _lib

_lib.lib()
M, K, N = [int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (256, 2048, 512))]
x = torch.randn(M, K, device='cuda').bfloat16()
w = torch.randn(N, K, device='cuda').bfloat16()
b = torch.randn(N, device='cuda')
out = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
ref = torch.relu(x.float() @ w.float().t() + b)
cands = [(F.pick_tile(M, N), 1)] + [c for c in F._split_candidates(M, N, K) if 1 < c[1] <= 16]
for tile, s in cands:
    def run():
        if s == 1:
            F.igemm(F.KIND_DENSE, 0, x, w, out, M, N, K, K, K, N, bias=b, flags=F.FLAG_BIAS | F.FLAG_RELU, tile=tile)
        else:
            slab = torch.empty((s, M, N), device='cuda')
            F.igemm(F.KIND_DENSE, 1, x, w, slab, M, N, K, K, K, N, splits=s, slab_stride=M * N, tile=tile)
            _lib.call("rk_reduce_slabs_epi", F._p(slab), s, M, N, F._p(b), 1, 0.2, 1.0, F._p(out), None, N, F._s())
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run()
    e1.record()
    e1.synchronize()
    err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
    print('tile %3d splits %3d  %7.2f us  err %.2e' % (tile, s, e0.elapsed_time(e1) / 20 * 1e3, err))
# graph-timed (what the autotuner now measures)
from rafiki_amd.ops import autotune
for tile, s in cands[:6]:
    def run(cfg):
        t, sp = cfg
        if sp == 1:
            F.igemm(F.KIND_DENSE, 0, x, w, out, M, N, K, K, K, N, bias=b, flags=F.FLAG_BIAS | F.FLAG_RELU, tile=t)
        else:
            slab = torch.empty((sp, M, N), device='cuda')
            F.igemm(F.KIND_DENSE, 1, x, w, slab, M, N, K, K, K, N, splits=sp, slab_stride=M * N, tile=t)
            _lib.call("rk_reduce_slabs_epi", F._p(slab), sp, M, N, F._p(b), 1, 0.2, 1.0, F._p(out), None, N, F._s())
    print('graph-timed tile %3d splits %3d  %7.2f us' % (tile, s, autotune._time_graph((tile, s), run, 10) * 1e3))
