# One image for every rafiki_amd process (admin, advisor, train/inference workers, predictor) on an
# MI355X node.  Replaces the reference's five images (dockerfiles/{admin,advisor,predictor,worker,
# admin_web}.Dockerfile); the worker image's CUDA 9 / cuDNN / NCCL stack is ROCm + RCCL here.
#
#   docker build -f dockerfiles/rafiki_amd.Dockerfile -t rafiki_amd .
#   docker run --device=/dev/kfd --device=/dev/dri --group-add video --ipc=host --network=host \
#       -e HSA_ENABLE_IPC_MODE_LEGACY=0 -v $PWD/data:/root/rafiki/data rafiki_amd            # admin
#   docker run ... rafiki_amd python -m rafiki_amd.worker                                      # worker
#
# The base image must carry ROCm >= 7.0 and a PyTorch-ROCm build (the kernels are compiled for
# gfx950 at image build time; the container needs the GPUs only at run time).
ARG BASE=rocm/pytorch:latest
FROM ${BASE}

ENV HSA_ENABLE_IPC_MODE_LEGACY=0 \
    PYTORCH_ROCM_ARCH=gfx950 \
    RAFIKI_OFFLOAD_ARCH=gfx950 \
    PYTHONUNBUFFERED=1

WORKDIR /root/rafiki
# Python dependencies beyond torch: all optional paths degrade gracefully when absent
RUN pip install --no-cache-dir numpy scipy scikit-learn pillow requests pyyaml

COPY rafiki_amd/ rafiki_amd/
COPY rafiki/ rafiki/
COPY csrc/ csrc/
COPY scripts/ scripts/
COPY examples/ examples/
COPY env.sh __graft_entry__.py bench.py ./

# hipcc --offload-arch=gfx950 kernels + g++ host runtime, in-tree
RUN python -m rafiki_amd._build

EXPOSE 3000 3002 3003
CMD ["python", "-m", "rafiki_amd.admin"]
