"""BiLSTM fwd+bwd time: gfx950 persistent-recurrence kernels vs torch nn.LSTM (MIOpen) on the same
GPU, PyBiLstm-shaped batches (PTB POS tagging: batch 16..128, sentence length ~25-60), plus the whole
tagger training step (embedding gather -> BiLSTM -> output layer -> cross-entropy -> backward -> Adam) on
the in-tree kernels.  Prints one JSON line.
usage: python scripts/dev/bench_lstm.py [--reps 20] [--only-tagger]   (rocprofv3 --stats over --only-tagger:
the per-kernel list of the tagger step, which should hold no hipBLASLt Cijk_* / MIOpen GEMM)"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch


def tagger_step(reps, B=128, T=40, V=20000, E=64, H=128, tags=48):
    """One PyBiLstm training step (rafiki_amd/models/pos_tagging.py Net, fp32) on a B x T batch."""
    import torch.nn.functional as F
    from rafiki_amd.ops.autograd import dense
    from rafiki_amd.ops.lstm import bilstm, embedding
    torch.manual_seed(0)
    emb = torch.nn.Embedding(V, E, padding_idx=0).cuda()
    lstm = torch.nn.LSTM(E, H, batch_first=True, bidirectional=True).cuda()
    out = torch.nn.Linear(2 * H, tags).cuda()
    params = list(emb.parameters()) + list(lstm.parameters()) + list(out.parameters())
    opt = torch.optim.Adam(params, lr=1e-3)
    x = torch.randint(1, V, (B, T), device='cuda')
    y = torch.randint(0, tags, (B, T), device='cuda')

    def step():
        h = bilstm(embedding(x, emb), lstm, dtype='fp32')
        logits = dense(h.reshape(-1, 2 * H), out.weight, out.bias)
        loss = F.cross_entropy(logits, y.reshape(-1))
        opt.zero_grad()
        loss.backward()
        opt.step()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / reps
    return {'B': B, 'T': T, 'V': V, 'E': E, 'H': H, 'tags': tags, 'ms_per_step': round(ms, 3),
            'tokens_per_s': round(B * T / ms * 1e3, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--only-tagger', action='store_true')
    a = ap.parse_args()
    from rafiki_amd.ops import _lib
    from rafiki_amd.ops.lstm import bilstm
    _lib.lib()
    res = {'metric': 'BiLSTM fwd+bwd ms (1 layer, bidirectional)', 'cases': []}
    res['tagger_step'] = tagger_step(a.reps)
    for B, T, E, H in ([] if a.only_tagger else [(32, 40, 64, 64), (128, 40, 64, 128), (128, 60, 128, 128)]):
        lstm = torch.nn.LSTM(E, H, batch_first=True, bidirectional=True).cuda()
        x = torch.randn(B, T, E, device='cuda', requires_grad=True)
        gy = torch.randn(B, T, 2 * H, device='cuda')
        row = {'B': B, 'T': T, 'E': E, 'H': H}
        for name, fn in (('rafiki_hip_fp32', lambda: bilstm(x, lstm, dtype='fp32')),
                         ('rafiki_hip_bf16', lambda: bilstm(x, lstm, dtype='bf16')),
                         ('torch_miopen', lambda: lstm(x)[0])):
            for _ in range(3):
                (fn() * gy).sum().backward()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                (fn() * gy).sum().backward()
            torch.cuda.synchronize()
            row[name + '_ms'] = round((time.perf_counter() - t0) * 1e3 / a.reps, 3)
        row['speedup_fp32'] = round(row['torch_miopen_ms'] / row['rafiki_hip_fp32_ms'], 2)
        row['speedup_bf16'] = round(row['torch_miopen_ms'] / row['rafiki_hip_bf16_ms'], 2)
        res['cases'].append(row)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
