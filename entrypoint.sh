#!/bin/bash
# Container entrypoint -- same env contract as the reference's entrypoint.sh:
#   NF_DISCOVERY_SERVICE (required)  headless service for peer DNS
#   REPLICAS             (required)  number of nodes
#   NPROC_PER_NODE       (default 1) workers per node (8 on an MI355X node)
#   MASTER_PORT          (default 29500)
#   TRAINING_SCRIPT      (default train.py)
#   SCRIPT_ARGS          extra args, word-split
# Node rank comes from the StatefulSet-style hostname suffix "<base>-<k>" and
# the master is "<base>-0.<service>".  Launches one process per GPU through
# the framework's torchrun-compatible launcher (LAUNCHER=torchrun to use torchrun).
set -e

MASTER_PORT=${MASTER_PORT:-29500}
NPROC_PER_NODE=${NPROC_PER_NODE:-1}
TRAINING_SCRIPT=${TRAINING_SCRIPT:-train.py}
HEADLESS_SERVICE="${NF_DISCOVERY_SERVICE}"
LAUNCHER=${LAUNCHER:-dpe}

log() {
    echo "[$(date -u +%H:%M:%S)] $1"
}

if [ -z "${HEADLESS_SERVICE}" ]; then
    log "ERROR: NF_DISCOVERY_SERVICE not set"
    exit 1
fi

if [ -z "${REPLICAS}" ]; then
    log "ERROR: REPLICAS not set"
    exit 1
fi

HOSTNAME=$(hostname)
NODE_RANK=${HOSTNAME##*-}
BASE_NAME=${HOSTNAME%-*}
case "${NODE_RANK}" in
    ''|*[!0-9]*)
        if [ "${REPLICAS}" = "1" ]; then
            NODE_RANK=0
        else
            log "ERROR: hostname '${HOSTNAME}' has no numeric '-<k>' suffix; cannot derive the node rank"
            exit 1
        fi
        ;;
esac
if [ "${REPLICAS}" = "1" ] && [ -z "${MASTER_ADDR}" ]; then
    MASTER_ADDR=127.0.0.1
else
    MASTER_ADDR=${MASTER_ADDR:-"${BASE_NAME}-0.${HEADLESS_SERVICE}"}
fi

export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}

log "Node ${NODE_RANK}/${REPLICAS} starting, master=${MASTER_ADDR}"
log "Starting launcher (rendezvous will synchronize nodes)"

if [ "${LAUNCHER}" = "torchrun" ]; then
    exec torchrun \
        --nnodes=${REPLICAS} \
        --nproc-per-node=${NPROC_PER_NODE} \
        --node-rank=${NODE_RANK} \
        --master-addr=${MASTER_ADDR} \
        --master-port=${MASTER_PORT} \
        ${TRAINING_SCRIPT} ${SCRIPT_ARGS}
fi
exec python3 -m distributed_pytorch_example_amd.launch \
    --nnodes=${REPLICAS} \
    --nproc-per-node=${NPROC_PER_NODE} \
    --node-rank=${NODE_RANK} \
    --master-addr=${MASTER_ADDR} \
    --master-port=${MASTER_PORT} \
    ${TRAINING_SCRIPT} ${SCRIPT_ARGS}
