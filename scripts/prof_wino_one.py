"""One Winograd conv shape in a loop (for rocprofv3 PMC passes): python scripts/prof_wino_one.py N H C K reps"""
import sys

sys.path.insert(0, '.')
import torch

from rafiki_amd.ops import _lib, f32 as S

N, H, C, K, reps = (int(v) for v in sys.argv[1:6])
_lib.lib()
x = torch.randn(N, H, H, C, device='cuda')
w = torch.randn(K, 9 * C, device='cuda') * 0.05
u = torch.empty(16, K, C, device='cuda')
S.wino_weights(w, u)
acc = torch.zeros((S.bn_slots(K), 2, K), dtype=torch.float64, device='cuda')
for _ in range(reps):
    S.wino_conv(x, u, stats=acc)
torch.cuda.synchronize()
