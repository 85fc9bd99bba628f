"""Tagger training-step timing / kernel census (K18): PyBiLstm at E=37, H=51, 45 tags on the native
engine, batches of 32 sentences bucketed by length.  Prints one JSON line (ms/step, tokens/s).
Run under ``rocprofv3 --kernel-trace --stats`` for the step's kernel list."""
import argparse
import json
import time

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from rafiki_amd.engine.tagger import TaggerEngine


class Net(torch.nn.Module):
    def __init__(self, V, E, H, NT):
        super().__init__()
        self.emb = torch.nn.Embedding(V, E, padding_idx=0)
        self.lstm = torch.nn.LSTM(E, H, batch_first=True, bidirectional=True)
        self.out = torch.nn.Linear(2 * H, NT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--E', type=int, default=37)
    ap.add_argument('--H', type=int, default=51)
    ap.add_argument('--tags', type=int, default=45)
    ap.add_argument('--V', type=int, default=20000)
    ap.add_argument('--B', type=int, default=32)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--graph', type=int, default=1)
    a = ap.parse_args()
    torch.manual_seed(0)
    net = Net(a.V, a.E, a.H, a.tags).cuda()
    eng = TaggerEngine(net, lr=0.05, dropout=0.1, seed=1)
    rng = np.random.default_rng(0)
    lengths = [8, 12, 16, 20, 24, 28, 32, 40]        # bucket lengths of a PTB-like corpus
    batches = []
    for L in lengths:
        x = rng.integers(1, a.V, (a.B, L))
        y = rng.integers(0, a.tags, (a.B, L))
        batches.append((x, y))
    for x, y in batches * 2:                          # eager + capture per shape, then one replay
        eng.step(x, y, graph=bool(a.graph))
    torch.cuda.synchronize()
    eng.take_loss()
    t0 = time.perf_counter()
    toks = 0
    for i in range(a.steps):
        x, y = batches[i % len(batches)]
        eng.step(x, y, graph=bool(a.graph))
        toks += x.size
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({'what': 'tagger_step', 'E': a.E, 'H': a.H, 'tags': a.tags, 'B': a.B, 'graph': a.graph,
                      'ms_per_step': round(1e3 * dt / a.steps, 4), 'tokens_per_s': round(toks / dt, 1),
                      'loss': eng.take_loss() / a.steps}))


if __name__ == '__main__':
    main()
