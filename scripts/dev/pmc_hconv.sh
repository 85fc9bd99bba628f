# PMC counters of the halo conv vs the implicit GEMM on the 32x32x64 VGG layer (forward)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmch
for t in 65 h0g512 h0g0; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmch/a$t -o run -- python3 scripts/dev/prof_one.py 1 fwd $t 5 > /dev/null
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d gpurun_out/pmch/b$t -o run -- python3 scripts/dev/prof_one.py 1 fwd $t 5 > /dev/null
done
echo ok
