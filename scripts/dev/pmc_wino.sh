#!/bin/bash
# PMC passes over one Winograd conv shape: scripts/dev/pmc_wino.sh <tag> N H C K [fwd|wgrad [splits]]
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA \
  SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/p0 -o run -- python3 scripts/dev/prof_wino_one.py $1 $2 $3 $4 8 $5 $6 > $OUT/p0.log 2>&1
python3 scripts/dev/pmc_kernel_avg.py $OUT/p0 --match wino > $OUT/summary.txt
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU \
  SQ_WAIT_INST_LDS SQ_INSTS_VMEM TA_BUSY_avr GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/p1 -o run -- python3 scripts/dev/prof_wino_one.py $1 $2 $3 $4 8 $5 $6 > $OUT/p1.log 2>&1
python3 scripts/dev/pmc_kernel_avg.py $OUT/p1 --match wino >> $OUT/summary.txt
rm -rf $OUT/p0 $OUT/p1
cat $OUT/summary.txt
