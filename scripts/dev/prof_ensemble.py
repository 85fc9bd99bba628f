"""Kernel timeline of one-graph ensemble replays (run under rocprofv3 --kernel-trace), or analyse it.

  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pe -o run -- python3 scripts/dev/prof_ensemble.py --batch 1
  python3 scripts/dev/prof_ensemble.py --analyze <kernel_trace.csv> --replays 20
"""
import argparse
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(a):
    import numpy as np
    import torch
    from rafiki_amd.predictor.predictor import Predictor
    from bench_predictor import build_models
    dev = torch.device('cuda', 0)
    models = build_models(a.models, dev)
    p = Predictor(models)
    arr = np.random.default_rng(0).integers(0, 256, (a.batch, 32, 32, 3), dtype=np.uint8)
    for _ in range(5):
        p.predict_array(arr)
    torch.cuda.synchronize()
    for _ in range(a.replays):
        p.predict_array(arr)
    torch.cuda.synchronize()


def analyze(path, replays):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    # split into replays at gaps > 50 us between consecutive kernel starts
    groups, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[0] - max(x[1] for x in cur) > 50_000:
            groups.append(cur)
            cur = [r]
        else:
            cur.append(r)
    groups.append(cur)
    last = groups[-replays:]
    spans = [(g[-1][1] if g else 0) - g[0][0] for g in last]
    spans = [max(x[1] for x in g) - g[0][0] for g in last]
    busy = [sum(x[1] - x[0] for x in g) for g in last]
    n = [len(g) for g in last]
    print('replays analysed {}  kernels/replay {}  span us (median) {:.1f}  sum of kernel us {:.1f}  '
          'concurrency {:.2f}'.format(len(last), n[len(n) // 2], sorted(spans)[len(spans) // 2] / 1e3,
                                      sorted(busy)[len(busy) // 2] / 1e3,
                                      sorted(busy)[len(busy) // 2] / max(1, sorted(spans)[len(spans) // 2])))
    # gaps between consecutive kernels (launch/dependency latency)
    g = last[-1]
    gaps = [max(0, g[i + 1][0] - g[i][1]) for i in range(len(g) - 1)]
    print('median inter-kernel gap us {:.2f}  total gap us {:.1f}'.format(sorted(gaps)[len(gaps) // 2] / 1e3,
                                                                         sum(gaps) / 1e3))
    by = collections.defaultdict(list)
    for gg in last:
        for s, e, name in gg:
            by[name[:90]].append(e - s)
    tot = sum(sum(v) for v in by.values()) / len(last)
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:25]:
        print('{:10.1f} us/replay {:5.1f}%  n/replay {:5.1f}  {}'.format(sum(v) / len(last) / 1e3,
                                                                      100 * sum(v) / len(last) / tot,
                                                                      len(v) / len(last), name))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=1)
    ap.add_argument('--models', type=int, default=4)
    ap.add_argument('--replays', type=int, default=20)
    ap.add_argument('--analyze', default='')
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze, a.replays)
    else:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        run(a)


if __name__ == '__main__':
    main()
