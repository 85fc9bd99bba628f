"""One Winograd conv shape in a loop (for rocprofv3 PMC passes):
python scripts/dev/prof_wino_one.py N H C K reps [fwd|wgrad|fwd4|wgrad4 [splits | variant]]"""
import sys

sys.path.insert(0, '.')
import torch

from rafiki_amd.ops import _lib, f32 as S

N, H, C, K, reps = (int(v) for v in sys.argv[1:6])
mode = sys.argv[6] if len(sys.argv) > 6 else 'fwd'
_lib.lib()
x = torch.randn(N, H, H, C, device='cuda')
if mode == 'wgrad4':
    dy = torch.randn(N, H, H, K, device='cuda')
    dw = torch.empty(K, 9 * C, device='cuda')
    splits = int(sys.argv[7]) if len(sys.argv) > 7 else S._wino4_wgrad_cands(N, H, H, K, C)[-1][2]
    for _ in range(reps):
        S.wino4_wgrad(dy, x, dw, splits=splits)
elif mode == 'fwd4':
    w = torch.randn(K, 9 * C, device='cuda') * 0.05
    u4 = S.wino4_u(w)
    acc = torch.zeros((S.bn_slots(K), 2, K), dtype=torch.float64, device='cuda')
    variant = int(sys.argv[7]) if len(sys.argv) > 7 else 0
    for _ in range(reps):
        S.wino4_conv(x, u4, stats=acc, variant=variant)
elif mode == 'wgrad':
    dy = torch.randn(N, H, H, K, device='cuda')
    dw = torch.empty(K, 9 * C, device='cuda')
    splits = int(sys.argv[7]) if len(sys.argv) > 7 else S._wino_wgrad_cands(N, H, H, K, C)[-1][2]
    for _ in range(reps):
        S.wino_wgrad(dy, x, dw, splits=splits)
else:
    w = torch.randn(K, 9 * C, device='cuda') * 0.05
    u = torch.empty(16, K, C, device='cuda')
    S.wino_weights(w, u)
    acc = torch.zeros((S.bn_slots(K), 2, K), dtype=torch.float64, device='cuda')
    for _ in range(reps):
        S.wino_conv(x, u, stats=acc)
torch.cuda.synchronize()
