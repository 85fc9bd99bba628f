# Hardware counters of single x6p GEMM configs (bench_x6p.py shapes, plain launches):
#   bash scripts/dev/pmc_x6p.sh <shape> <cfg> [dbg]   e.g.  pmc_x6p.sh c5f 3,2,1 1
# -> gpurun_out/pmc_x6p/<shape>_<cfg>_<dbg>.txt: per-dispatch averages of MFMA busy, waits, LDS, clock
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
S=$1; C=$2; D=${3:-0}
O=gpurun_out/pmc_x6p; T=$O/${S}_${C//,/-}_$D
mkdir -p $O
export X6P_SHAPES=$S X6P_CFGS=$C X6P_EAGER=1 RAFIKI_X6P_DBG=$D
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA \
  SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $T.p0 -o run -- \
  python3 scripts/dev/bench_x6p.py > $T.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $T.p1 -o run -- \
  python3 scripts/dev/bench_x6p.py >> $T.log 2>&1
python3 - "$T" > $T.txt <<'PY'
import csv, glob, sys, collections
T = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter(); dur = []
for d in (T + '.p0', T + '.p1'):
    for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            if 'x6p_' not in r['Kernel_Name']:
                continue
            tot[r['Counter_Name']] += float(r['Counter_Value'])
            if (d, r['Dispatch_Id']) not in seen:
                seen.add((d, r['Dispatch_Id'])); n[d] += 1
    for f in glob.glob(d + '/**/*kernel_trace.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'x6p_' in r['Kernel_Name']:
                dur.append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-3)
k0 = max(1, n[T + '.p0'])
avg = {c: v / k0 for c, v in tot.items()}
g = avg.get('GRBM_GUI_ACTIVE', 1)
print('dispatches', dict(n), 'mean us (perturbed)', round(sum(dur) / max(1, len(dur)), 2))
for c in sorted(avg):
    print('%-28s %14.0f' % (c, avg[c]))
print('MfmaUtil% (MFMA_BUSY / (GUI_ACTIVE * 1024 SIMDs))', round(100 * avg.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (g * 1024), 1))
print('MFMA busy cycles per MFMA instr', round(avg.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(1, avg.get('SQ_INSTS_MFMA', 1)), 2))
print('GUI_ACTIVE / traced us (MHz, perturbed)', round(g / max(1e-9, sum(dur) / max(1, len(dur))), 1))
PY
rm -rf $T.p0 $T.p1
cat $T.txt
