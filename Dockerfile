# MI355X (gfx950) image: ROCm PyTorch base, framework built in-tree for gfx950.
# Same runtime contract as the reference image: ENTRYPOINT ./entrypoint.sh with
# REPLICAS / MASTER_PORT / NPROC_PER_NODE defaults.  Run on one 8-GPU node:
#   docker run --device=/dev/kfd --device=/dev/dri --group-add video --ipc=host \
#     --hostname job-0 -e NF_DISCOVERY_SERVICE=local -e REPLICAS=1 -e NPROC_PER_NODE=8 <image>
# Pinned base (the reference pins pytorch/pytorch:2.9.1-cuda12.6-cudnn9-runtime, Dockerfile:1): the stack
# this repository is built and measured on -- PyTorch 2.10.0 built for ROCm 7.0 (torch-bundled HIP 7.0 /
# RCCL 2.26), Python 3.10, Ubuntu 22.04.  Override with --build-arg BASE_IMAGE=... to move deliberately;
# the extension links torch's own libamdhip64 / librccl, so the image's torch is the ABI that matters.
ARG BASE_IMAGE=rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.10.0
FROM ${BASE_IMAGE}

ENV DEBIAN_FRONTEND=noninteractive
ENV PYTHONUNBUFFERED=1
ENV PYTORCH_ROCM_ARCH=gfx950
ENV HSA_ENABLE_IPC_MODE_LEGACY=0

WORKDIR /workspace

COPY distributed_pytorch_example_amd/ distributed_pytorch_example_amd/
COPY csrc/ csrc/
COPY train.py bench.py entrypoint.sh __graft_entry__.py ./

RUN python3 -m distributed_pytorch_example_amd._build && chmod +x entrypoint.sh

ENV REPLICAS=2
ENV MASTER_PORT=29500
ENV NPROC_PER_NODE=1

ENTRYPOINT ["./entrypoint.sh"]
