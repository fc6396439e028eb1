# Rehearse the driver's multi-rank bench path on a 1-GPU box: two bench.py ranks share GPU 0
# (LOCAL_RANK=0 for both, distinct NCCL_HOSTID so RCCL uses its socket transport), real RCCL
# all-reduces of the DDP buckets at world 2.  Throughput here says nothing about xGMI.
set -o pipefail
mkdir -p gpurun_out
PORT=$((29500 + RANDOM % 1000))
for model in resnet50 gpt2; do
  pids=()
  for r in 0 1; do
    RANK=$r WORLD_SIZE=2 LOCAL_RANK=0 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
    NCCL_HOSTID=dpe-bench-host-$r NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 OMP_NUM_THREADS=1 \
    timeout -k 10 400 python -u bench.py --gpus 2 --model $model --steps 6 --warmup 3 \
        $([ $model = resnet50 ] && echo "--batch-size 128" || echo "--batch-size 4") > gpurun_out/w2_$model.$r.log 2>&1 &
    pids+=($!)
  done
  rc=0
  for p in "${pids[@]}"; do wait $p || rc=$?; done
  [ $rc -ne 0 ] && { tail -20 gpurun_out/w2_$model.0.log gpurun_out/w2_$model.1.log; exit $rc; }
  tail -1 gpurun_out/w2_$model.0.log | cut -c1-260
  PORT=$((PORT + 1))
done
