#!/bin/bash
# round-5 final evidence on the shipped tune DB: GPU suite + smoke + default bench, the VGG-small step
# kernels + PMC, PG-GAN lod 3 / lod 0 kernels + PMC
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_final.sh || exit 1
bash scripts/gpu_final.sh prof || exit 1
timeout -k 10 600 bash scripts/gpu_pggan_prof.sh 3 6 > gpurun_out/pgprof3.log 2>&1 || { tail -5 gpurun_out/pgprof3.log; exit 1; }
head -2 gpurun_out/pgprof_lod3/kernels.txt
timeout -k 10 600 bash scripts/gpu_pggan_prof.sh 0 3 > gpurun_out/pgprof0.log 2>&1 || { tail -5 gpurun_out/pgprof0.log; exit 1; }
head -2 gpurun_out/pgprof_lod0/kernels.txt
