"""Drive one halo-conv forward config (VGG-small layer 2: 32x32, 64->64, batch 256) N times for a
rocprofv3 --pmc pass (scripts/dev/pmc_hconv.sh covers the step-level counters)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from rafiki_amd.ops import functional as F

B, hw, cin, cout = 256, 32, 64, 64
x = torch.randn(B, hw, hw, cin, device='cuda').bfloat16()
w = (torch.randn(cout, 9 * cin, device='cuda') * 0.05).bfloat16()
y = torch.empty(B, hw, hw, cout, device='cuda', dtype=torch.bfloat16)
M, K = B * hw * hw, 9 * cin
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    F.hconv(0, x, w, y, M, cout, K, K, hw, hw, cin, bn_bit=0, grid=512)
torch.cuda.synchronize()
