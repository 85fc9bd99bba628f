"""BiLSTM fwd+bwd time: gfx950 persistent-recurrence kernels vs torch nn.LSTM (MIOpen) on the same
GPU, PyBiLstm-shaped batches (PTB POS tagging: batch 16..128, sentence length ~25-60).
Prints one JSON line.  usage: python scripts/bench_lstm.py [--reps 20]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=20)
    a = ap.parse_args()
    from rafiki_amd.ops import _lib
    from rafiki_amd.ops.lstm import bilstm
    _lib.lib()
    res = {'metric': 'BiLSTM fwd+bwd ms (1 layer, bidirectional)', 'cases': []}
    for B, T, E, H in [(32, 40, 64, 64), (128, 40, 64, 128), (128, 60, 128, 128)]:
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
