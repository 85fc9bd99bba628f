"""Per-kernel hardware-counter summary of steady-state training steps.

Reads the ``counter_collection.csv`` files of several rocprofv3 ``--pmc`` passes over the same
program (``scripts/pmc_step.sh``), keeps the dispatches of the last K steps (the trace is cut at
the optimizer kernel that ends every step, as in ``trace_steps.py``) and aggregates per kernel:

* ``mfma_util_pct``  = sum SQ_VALU_MFMA_BUSY_CYCLES / (kernel cycles * 1024 SIMDs) * 100 (the
  rocprofiler-sdk ``MfmaUtil`` expression).  Counter collection serialises dispatches and stretches
  GRBM_GUI_ACTIVE far past the kernel, so the kernel cycles come from an unperturbed kernel trace
  of the same run (``--durations``, a ``trace_steps.py --csv`` file) at the 2.4 GHz peak clock;
  without it GRBM_GUI_ACTIVE is used (a lower bound)
* ``lds_conflict_pct`` = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE * 100 (extra cycles / LDS cycles)
* ``fetch_MB`` / ``write_MB`` = FETCH_SIZE / WRITE_SIZE (KB) per step; NOTE gfx950 FETCH_SIZE
  counts wide coalesced reads at half their bytes (MI355X_MICROARCH.md, HBM section), so the
  read side is a lower bound
* ``l2_hit_pct`` = TCC_HIT / (TCC_HIT + TCC_MISS)

usage: python scripts/pmc_summary.py <pass_dir> [<pass_dir> ...] --steps K [--csv out.csv]
"""
import argparse
import collections
import csv
import glob
import os
import re


def short(name):
    name = re.sub(r'\(anonymous namespace\)::', '', name)
    m = re.match(r'(?:void )?([\w:<>, ]+?)\(', name)
    return (m.group(1) if m else name)[:90]


def load_pass(d, steps, marker):
    files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    if not files:
        raise SystemExit('no counter_collection.csv under %s' % d)
    disp = collections.OrderedDict()     # dispatch id -> (name, {counter: value})
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                did = int(r['Dispatch_Id'])
                ent = disp.setdefault(did, [r['Kernel_Name'], collections.defaultdict(float)])
                ent[1][r['Counter_Name']] += float(r['Counter_Value'])
    order = sorted(disp)
    ends = [i for i, did in enumerate(order) if marker in disp[did][0]]
    # the marker may launch several times per step (one per parameter range): a step ends at the
    # last launch of each consecutive group (same rule as trace_steps.py)
    marks = [e for j, e in enumerate(ends) if j + 1 == len(ends) or ends[j + 1] != e + 1]
    if len(marks) < steps + 1:
        raise SystemExit('%s: only %d step markers' % (d, len(marks)))
    lo, hi = marks[-steps - 1] + 1, marks[-1] + 1
    return [disp[did] for did in order[lo:hi]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('passes', nargs='+')
    ap.add_argument('--steps', type=int, default=2)
    ap.add_argument('--marker', default='sgd_kernel')
    ap.add_argument('--csv', default='')
    ap.add_argument('--durations', default='', help='trace_steps.py --csv output of an unprofiled run')
    ap.add_argument('--ghz', type=float, default=2.4)
    a = ap.parse_args()
    dur = {}
    if a.durations:
        with open(a.durations) as f:
            dur = {r['kernel']: float(r['us_per_step']) for r in csv.DictReader(f)}
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.Counter()
    for pi, d in enumerate(a.passes):
        for name, ctr in load_pass(d, a.steps, a.marker):
            k = short(name)
            if pi == 0:
                launches[k] += 1
            for c, v in ctr.items():
                if c == 'GRBM_GUI_ACTIVE':
                    agg[k]['GRBM_GUI_ACTIVE@%d' % pi] += v
                else:
                    agg[k][c] += v
    rows = []
    tot = collections.defaultdict(float)
    for k, c in agg.items():
        gui = c.get('GRBM_GUI_ACTIVE@0', 0.0)
        r = {'kernel': k, 'launches_per_step': launches[k] / a.steps, 'us_per_step': dur.get(k, '')}
        cyc = dur[k] * 1e3 * a.ghz * a.steps if k in dur else gui
        if 'SQ_VALU_MFMA_BUSY_CYCLES' in c and cyc:
            r['mfma_util_pct'] = round(100.0 * c['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024), 2)
        if k in dur and dur[k] > 0 and ('FETCH_SIZE' in c or 'WRITE_SIZE' in c):
            r['GBps'] = round((c.get('FETCH_SIZE', 0) + c.get('WRITE_SIZE', 0)) * 1024 / a.steps / (dur[k] * 1e3), 1)
        if c.get('SQ_LDS_IDX_ACTIVE'):
            r['lds_conflict_pct'] = round(100.0 * c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_LDS_IDX_ACTIVE'], 2)
        if 'FETCH_SIZE' in c:
            r['fetch_MB'] = round(c['FETCH_SIZE'] / 1024 / a.steps, 2)
        if 'WRITE_SIZE' in c:
            r['write_MB'] = round(c['WRITE_SIZE'] / 1024 / a.steps, 2)
        h, m = c.get('TCC_HIT_sum', 0), c.get('TCC_MISS_sum', 0)
        if h + m:
            r['l2_hit_pct'] = round(100.0 * h / (h + m), 1)
        wc = c.get('SQ_WAVE_CYCLES', 0)
        if wc:   # shares of wave lifetime: parked (waitcnt / barrier), issue-stalled, issuing VALU
            r['wait_pct'] = round(100.0 * c.get('SQ_WAIT_ANY', 0) / wc, 1)
            if 'SQ_WAIT_INST_ANY' in c:
                r['stall_pct'] = round(100.0 * c['SQ_WAIT_INST_ANY'] / wc, 1)
            if 'SQ_ACTIVE_INST_VALU' in c:
                r['valu_pct'] = round(100.0 * c['SQ_ACTIVE_INST_VALU'] / wc, 1)
        if c.get('SQ_INSTS_MFMA') and 'SQ_INSTS_VALU' in c:
            r['valu_per_mfma'] = round(c['SQ_INSTS_VALU'] / c['SQ_INSTS_MFMA'], 2)
        r['gui_kcycles_per_step'] = round(gui / 1e3 / a.steps, 1)
        for key in ('SQ_VALU_MFMA_BUSY_CYCLES', 'FETCH_SIZE', 'WRITE_SIZE'):
            tot[key] += c.get(key, 0)
        tot['gui'] += gui
        tot['cyc'] += cyc
        rows.append(r)
    rows.sort(key=lambda r: -(r['us_per_step'] or 0) * 1e6 - r['gui_kcycles_per_step'])
    cols = ['kernel', 'launches_per_step', 'us_per_step', 'mfma_util_pct', 'lds_conflict_pct',
            'fetch_MB', 'write_MB', 'GBps', 'l2_hit_pct', 'wait_pct', 'stall_pct', 'valu_pct', 'valu_per_mfma']
    print(('%-60s' + '%11s' * (len(cols) - 1)) % tuple(c[:10] for c in cols))
    for r in rows:
        print(('%-60s' + '%11s' * (len(cols) - 1)) % tuple([r['kernel'][:60]] + [r.get(c, '') for c in cols[1:]]))
    if tot['gui']:
        print('step total: MfmaUtil %.2f%%  fetch %.1f MB  write %.1f MB  busy %.1f kcycles' % (
            100.0 * tot['SQ_VALU_MFMA_BUSY_CYCLES'] / (tot['cyc'] * 1024), tot['FETCH_SIZE'] / 1024 / a.steps,
            tot['WRITE_SIZE'] / 1024 / a.steps, tot['gui'] / 1e3 / a.steps))
    if a.csv:
        with open(a.csv, 'w', newline='') as f:
            w = csv.DictWriter(f, fieldnames=cols)
            w.writeheader()
            for r in rows:
                w.writerow({c: r.get(c, '') for c in cols})


if __name__ == '__main__':
    main()
