import torch, time, json
torch.backends.cuda.matmul.allow_tf32 = False
res = []
for (M, K, N, tag) in [(4096, 4608, 512, 'L8 fwd'), (4096, 2304, 512, 'L7 fwd'), (512, 4096, 4608, 'L8 wgrad'),
                       (16384, 2304, 256, 'L6 fwd'), (256, 16384, 2304, 'L6 wgrad'), (65536, 1152, 128, 'L4 fwd'),
                       (128, 65536, 1152, 'L4 wgrad'), (262144, 576, 64, 'L2 fwd'), (64, 262144, 576, 'L2 wgrad'),
                       (8192, 8192, 8192, 'big')]:
    a = torch.randn(M, K, device='cuda').bfloat16()
    b = torch.randn(K, N, device='cuda').bfloat16()
    for _ in range(5): c = a @ b
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20): c = a @ b
    g.replay(); torch.cuda.synchronize()
    t0 = time.perf_counter(); g.replay(); torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 20
    res.append((tag, M, K, N, round(dt * 1e6, 2), round(2 * M * N * K / dt / 1e12, 1)))
for r in res: print(r)
