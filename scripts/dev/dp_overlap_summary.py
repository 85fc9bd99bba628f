"""Summarise a rocprofv3 kernel trace of scripts/dev/pggan_dp_trace.py: how many RCCL kernels ran,
and how much of their time overlapped other (gradient / optimizer) kernels on the GPU.
usage: python scripts/dev/dp_overlap_summary.py <kernel_trace.csv> [--last N]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--last', type=int, default=0, help='only the last N RCCL kernels (steady state)')
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    comm = [r for r in rows if 'nccl' in r[2].lower() or 'rccl' in r[2].lower()]
    other = [r for r in rows if r not in comm]
    if a.last:
        comm = comm[-a.last:]
    tot = ov = 0
    n_ov = 0
    for s, e, _ in comm:
        tot += e - s
        o = 0
        for s2, e2, _ in other:
            if s2 >= e:
                break
            if e2 > s:
                o += min(e, e2) - max(s, s2)
        o = min(o, e - s)
        ov += o
        n_ov += o > 0
    names = sorted({r[2][:80] for r in comm})
    print('rccl kernels {}  busy {:.1f} us  overlapped with compute {:.1f} us ({:.0f}%)  kernels overlapping {}'.format(
        len(comm), tot / 1e3, ov / 1e3, 100.0 * ov / max(1, tot), n_ov))
    for n in names[:8]:
        print('  ', n)


if __name__ == '__main__':
    main()
