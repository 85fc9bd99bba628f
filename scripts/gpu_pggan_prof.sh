#!/bin/bash
# PG-GAN per-kernel steady-state time (kernel trace) + PMC passes (MFMA utilisation; HBM fetch; HBM write)
# at one LOD.
#   scripts/gpu_pggan_prof.sh <lod> [steps]  -> gpurun_out/pgprof_lod<lod>/{kernels.txt,kernels.csv,pmc.txt}
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LOD=${1:-0}
STEPS=${2:-6}
OUT=gpurun_out/pgprof_lod$LOD
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t -o run -- \
  python3 scripts/bench_pg_gan.py --lods $LOD --steps $STEPS --warmup 3 > $OUT/t.log 2>&1
python3 scripts/trace_steps.py $(find $OUT/t -name '*kernel_trace.csv' | head -1) --steps $STEPS \
  --marker lerp_ --csv $OUT/kernels.csv --seq $OUT/seq.txt > $OUT/kernels.txt
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/p0 -o run -- python3 scripts/bench_pg_gan.py --lods $LOD --steps 2 --warmup 1 \
  > $OUT/p0.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/p1 -o run -- python3 scripts/bench_pg_gan.py --lods $LOD --steps 2 --warmup 1 \
  > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/p2 -o run -- python3 scripts/bench_pg_gan.py --lods $LOD --steps 2 --warmup 1 \
  > $OUT/p2.log 2>&1
python3 scripts/pmc_summary.py $OUT/p0 $OUT/p1 $OUT/p2 --steps 2 --marker lerp_ --durations $OUT/kernels.csv \
  --csv $OUT/pmc.csv > $OUT/pmc.txt
rm -rf $OUT/t $OUT/p0 $OUT/p1 $OUT/p2
tail -1 $OUT/t.log | cut -c1-300
head -40 $OUT/kernels.txt
tail -3 $OUT/pmc.txt
