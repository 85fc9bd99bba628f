#!/bin/bash
# round-5 profiles: VGG-small step kernels + PMC (shipped tune database), PG-GAN lod 3 kernels + PMC
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
bash scripts/gpu_final.sh prof || exit 1
timeout -k 10 900 bash scripts/gpu_pggan_prof.sh 3 6 > gpurun_out/pgprof3.log 2>&1
rc=$?; echo "pg lod3 rc=$rc"; tail -5 gpurun_out/pgprof3.log
