"""Average rocprofv3 --pmc counters per dispatch of kernels matching a name filter.

usage: python scripts/dev/pmc_kernel_avg.py <pass_dir> [--match sgemm] [--skip 2]
Prints per kernel: dispatches, mean counters, and derived MFMA utilisation / effective clock when
SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE are present.
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('d')
    ap.add_argument('--match', default='')
    ap.add_argument('--skip', type=int, default=2, help='leading dispatches (warm-up) to drop per kernel')
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.d, '**', '*counter_collection.csv'), recursive=True)
    disp = collections.OrderedDict()
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                if a.match not in r['Kernel_Name']:
                    continue
                ent = disp.setdefault(int(r['Dispatch_Id']), [r['Kernel_Name'], collections.defaultdict(float)])
                ent[1][r['Counter_Name']] += float(r['Counter_Value'])
    by = collections.defaultdict(list)
    for did in sorted(disp):
        by[disp[did][0]].append(disp[did][1])
    # kernel durations of the same run (kernel_trace.csv), if collected: effective clock
    dur = collections.defaultdict(list)
    for fn in glob.glob(os.path.join(a.d, '**', '*kernel_trace.csv'), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                if a.match in r['Kernel_Name']:
                    dur[r['Kernel_Name']].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
    for name, lst in by.items():
        lst = lst[a.skip:] or lst
        keys = sorted({k for d in lst for k in d})
        mean = {k: sum(d.get(k, 0.0) for d in lst) / len(lst) for k in keys}
        print(name[:120])
        print('  dispatches', len(lst))
        for k in keys:
            print('  {:28s} {:16.1f}'.format(k, mean[k]))
        if 'SQ_VALU_MFMA_BUSY_CYCLES' in mean and 'GRBM_GUI_ACTIVE' in mean:
            cyc = mean['GRBM_GUI_ACTIVE'] / 8.0
            print('  mfma_util_pct (vs GRBM span) {:.1f}'.format(100.0 * mean['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024)))
        if dur.get(name) and 'GRBM_GUI_ACTIVE' in mean:
            d = sorted(dur[name])[len(dur[name]) // 2] * 1e-9
            print('  median_dispatch_us {:.1f}  effective_clock_GHz {:.3f}'.format(
                d * 1e6, mean['GRBM_GUI_ACTIVE'] / 8.0 / d / 1e9))
        if 'SQ_BUSY_CYCLES' in mean and 'GRBM_GUI_ACTIVE' in mean:
            print('  sq_busy / grbm_per_xcd {:.3f}'.format(mean['SQ_BUSY_CYCLES'] / (mean['GRBM_GUI_ACTIVE'] / 8.0)))


if __name__ == '__main__':
    main()
