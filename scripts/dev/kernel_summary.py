"""Per-kernel time summary of a rocprofv3 kernel trace, restricted to the steady state.

usage: python scripts/dev/kernel_summary.py <kernel_trace.csv> [--last-frac 0.5] [--top 30] [--csv out.csv]
Only dispatches that START in the last ``last-frac`` of the traced time span count (warm-up,
autotuning and graph capture sit at the front).  Prints total GPU-busy time, the per-kernel share,
and the number of dispatches.
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--last-frac', type=float, default=0.5)
    ap.add_argument('--top', type=int, default=30)
    ap.add_argument('--csv', default='')
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    t0, t1 = min(r[0] for r in rows), max(r[1] for r in rows)
    cut = t1 - (t1 - t0) * a.last_frac
    sel = [r for r in rows if r[0] >= cut]
    by = collections.defaultdict(lambda: [0, 0])
    for s, e, n in sel:
        by[n][0] += e - s
        by[n][1] += 1
    tot = sum(v[0] for v in by.values())
    span = max(r[1] for r in sel) - min(r[0] for r in sel)
    print('window {:.3f} ms  kernel time {:.3f} ms  dispatches {}'.format(span / 1e6, tot / 1e6, len(sel)))
    items = sorted(by.items(), key=lambda kv: -kv[1][0])
    for n, (t, c) in items[:a.top]:
        print('{:10.1f} us {:5.1f}%  n={:5d}  {}'.format(t / 1e3, 100.0 * t / tot, c, n[:110]))
    if a.csv:
        with open(a.csv, 'w', newline='') as f:
            w = csv.writer(f)
            w.writerow(['kernel', 'total_us', 'pct', 'dispatches'])
            for n, (t, c) in items:
                w.writerow([n, round(t / 1e3, 2), round(100.0 * t / tot, 2), c])


if __name__ == '__main__':
    main()
