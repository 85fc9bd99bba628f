import sys, math, json
sys.path.insert(0, '.')
import torch, torch.nn.functional as TF
from rafiki_amd.ops import f32 as S, _lib
_lib.lib()
torch.manual_seed(0)
for (N, H, C, K) in [(32, 32, 64, 64), (32, 16, 128, 128), (32, 8, 256, 256), (32, 4, 512, 512)]:
    x = torch.randn(N, H, H, C)
    w = torch.randn(K, 3, 3, C) / math.sqrt(9 * C)
    ref = TF.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    u = torch.empty(16, K, C, device='cuda')
    S.wino_weights(w.cuda().reshape(K, -1).contiguous(), u)
    yw = S.wino_conv(x.cuda(), u).double().cpu()
    yd = S.conv_fwd(x.cuda(), w.cuda()).double().cpu()
    y32 = TF.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1).double()
    f = lambda a: ((a - ref).norm() / ref.norm()).item()
    m = lambda a: ((a - ref).abs().max() / ref.abs().max()).item()
    print(json.dumps(dict(H=H, C=C, wino_fro=f(yw), direct_fro=f(yd), torch_cpu_fro=f(y32), wino_max=m(yw), direct_max=m(yd))))
