# MI355X (gfx950) image: ROCm PyTorch base, framework built in-tree for gfx950.
# Same runtime contract as the reference image: ENTRYPOINT ./entrypoint.sh with
# REPLICAS / MASTER_PORT / NPROC_PER_NODE defaults.  Run on one 8-GPU node:
#   docker run --device=/dev/kfd --device=/dev/dri --group-add video --ipc=host \
#     --hostname job-0 -e NF_DISCOVERY_SERVICE=local -e REPLICAS=1 -e NPROC_PER_NODE=8 <image>
FROM rocm/pytorch:latest

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
