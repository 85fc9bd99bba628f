"""Per-kernel time of the last K training steps from a rocprofv3 kernel_trace.csv.

The whole-run ``kernel_stats.csv`` also counts warm-up and autotuning launches; this isolates
steady-state steps by cutting the trace at the optimizer kernel that ends every step.
usage: python scripts/trace_steps.py <kernel_trace.csv> [--steps K] [--marker sgd_kernel] [--csv out.csv]
"""
import argparse
import collections
import csv
import re


def short(name):
    name = re.sub(r'\(anonymous namespace\)::', '', name)
    m = re.match(r'(?:void )?([\w:<>, ]+?)\(', name)
    return (m.group(1) if m else name)[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--marker', default='sgd_kernel')
    ap.add_argument('--csv', default='')
    ap.add_argument('--seq', default='', help='write the per-launch sequence of a step (mean over the steps)')
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'],
                         r.get('Grid_Size', r.get('Grid_Size_X', '')), r.get('Workgroup_Size', r.get('Workgroup_Size_X', ''))))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if a.marker in r[2]]
    # the marker may launch several times per step (one per parameter range): keep the last launch
    # of each consecutive group
    last = [e for j, e in enumerate(ends) if j + 1 == len(ends) or ends[j + 1] != e + 1]
    if len(last) <= a.steps:
        raise SystemExit('only {} steps in trace'.format(len(last)))
    lo, hi = last[-a.steps - 1] + 1, last[-1] + 1
    sel = rows[lo:hi]
    wall = sel[-1][1] - sel[0][0]
    agg = collections.defaultdict(lambda: [0, 0])
    for s, e, n, *_ in sel:
        agg[short(n)][0] += 1
        agg[short(n)][1] += e - s
    busy = sum(v[1] for v in agg.values())
    print('steps {}  wall/step {:.1f} us  busy/step {:.1f} us  launches/step {:.0f}'.format(
        a.steps, wall / a.steps / 1e3, busy / a.steps / 1e3, len(sel) / a.steps))
    out = sorted(agg.items(), key=lambda kv: -kv[1][1])
    for n, (c, t) in out:
        print('{:8.1f} us/step {:5.1f}%  x{:<4d} {}'.format(t / a.steps / 1e3, 100.0 * t / busy, c // a.steps, n))
    if a.seq:
        per = len(sel) // a.steps
        with open(a.seq, 'w') as f:
            for i in range(per):
                ts = [sel[k * per + i][1] - sel[k * per + i][0] for k in range(a.steps)]
                r = sel[i]
                f.write('{:3d} {:8.1f} us  grid {:>8} wg {:>4}  {}\n'.format(i, sum(ts) / len(ts) / 1e3, r[3], r[4],
                                                                         short(r[2])))
    if a.csv:
        with open(a.csv, 'w', newline='') as f:
            w = csv.writer(f)
            w.writerow(['kernel', 'launches_per_step', 'us_per_step', 'pct_busy'])
            for n, (c, t) in out:
                w.writerow([n, c / a.steps, round(t / a.steps / 1e3, 2), round(100.0 * t / busy, 2)])


if __name__ == '__main__':
    main()
