#!/bin/bash
# Rehearse the driver's N-rank bench on a 1-GPU box: N bench.py ranks share GPU 0 (LOCAL_RANK=0, distinct
# NCCL_HOSTID, so RCCL connects them with its socket transport), real RCCL all-reduces of the DDP buckets
# at world N.  Rank 0 runs under rocprofv3 --kernel-trace: the RCCL kernels' grid (= channel blocks),
# workgroup size and residency per bucket all-reduce are summarised (scripts/rccl_kernels.py).
# Throughput here says nothing about xGMI.  Usage: bash scripts/world_1gpu.sh N [model] [per-rank batch]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-8}; MODEL=${2:-resnet50}; BS=${3:-32}
OUT=$R/gpurun_out/w${N}_$MODEL
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PORT=$((29500 + RANDOM % 1000))
args="--gpus $N --model $MODEL --batch-size $BS --steps 6 --warmup 3"
pids=()
for r in $(seq 1 $((N - 1))); do
  RANK=$r WORLD_SIZE=$N LOCAL_RANK=0 LOCAL_WORLD_SIZE=$N MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
  NCCL_HOSTID=dpe-w-host-$r NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 OMP_NUM_THREADS=1 \
  timeout -k 10 400 python3 -u $R/bench.py $args > $OUT/r$r.log 2>&1 &
  pids+=($!)
done
RANK=0 WORLD_SIZE=$N LOCAL_RANK=0 LOCAL_WORLD_SIZE=$N MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
NCCL_HOSTID=dpe-w-host-0 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 OMP_NUM_THREADS=1 \
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 -u $R/bench.py $args > $OUT/r0.log 2>&1
rc=$?
for p in "${pids[@]}"; do wait $p || rc=$?; done
[ $rc -ne 0 ] && { tail -20 $OUT/r0.log $OUT/r1.log; exit $rc; }
grep "\"metric\"" $OUT/r0.log | tail -1 > $OUT/bench.json
f=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/rccl_kernels.py "$f" $OUT/bench.json > $OUT/rccl.txt && cat $OUT/rccl.txt
rm -f $f
