"""bf16-vs-fp32 convergence runs (tests/test_convergence_gpu.py's run()) over learning rates / repeats.

usage: python scripts/dev/convergence_sweep.py --lrs 0.02,0.01 --repeats 2 --out gpurun_out/conv_sweep.json
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), 'tests'))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import test_convergence_gpu as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lrs', default='0.02,0.01')
    ap.add_argument('--repeats', type=int, default=2)
    ap.add_argument('--out', default='')
    a = ap.parse_args()
    res = []
    for lr in [float(v) for v in a.lrs.split(',')]:
        for r in range(a.repeats):
            s = T.summarise(T.run(lr=lr))
            s.update(lr=lr, repeat=r)
            res.append(s)
            print(json.dumps({k: s[k] for k in ('lr', 'repeat', 'acc_fp32', 'acc_bf16', 'mean_window_gap',
                                                'max_window_gap', 'last_window_gap')}), flush=True)
    if a.out:
        with open(a.out, 'w') as f:
            json.dump(res, f, indent=1)


if __name__ == '__main__':
    main()
