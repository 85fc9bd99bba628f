# counters of the halo-tiled X6 conv vs the fused F(4x4) Winograd forward on one VGG-small layer
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_xc
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
  SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/p0 -o run -- python3 scripts/prof_xconv_one.py 1 > $OUT/p0.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM \
  SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o run -- python3 scripts/prof_xconv_one.py 1 > $OUT/p1.log 2>&1
python3 - <<'PY'
import csv, glob, collections
for d in ('p0', 'p1'):
    f = glob.glob('gpurun_out/pmc_xc/%s/**/*counter_collection.csv' % d, recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for r in rows:
        k = r['Kernel_Name'][:70]
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
    for k, v in agg.items():
        print(d, k, {c: '%.3g' % x for c, x in v.items()})
PY
rm -rf $OUT/p0 $OUT/p1
