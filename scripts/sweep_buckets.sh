#!/bin/bash
# Bucket-size sweep (BASELINE config 3, SURVEY §5.8 design point 6): ResNet-50 DDP
# throughput and all-reduce/backward overlap per bucket cap, on N GPUs of one node.
#   bash scripts/sweep_buckets.sh 8            (N=8; N=1 runs the RCCL path with --force-comm)
# One JSON line per bucket size goes to gpurun_out/sweep_buckets_N<N>.jsonl.
set -o pipefail
N=${1:-8}
OUT=gpurun_out/sweep_buckets_N${N}.jsonl
mkdir -p gpurun_out && : > $OUT
for MB in 5 10 25 50 100; do
  if [ "$N" = "1" ]; then
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --bucket-mb $MB --bucket-timing 1 --force-comm >> $OUT || exit $?
  else
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $((29700 + MB)) bench.py --gpus $N --steps 10 --warmup 3 --bucket-mb $MB --bucket-timing 1 >> $OUT || exit $?
  fi
  tail -1 $OUT | python -c "import json,sys; d=json.loads(sys.stdin.read()); b=d.get('buckets',{}); print(f\"bucket {d['config']['bucket_mb']} MB: {d['value']:.0f} {d['unit']}, {b.get('count')} buckets, comm {b.get('comm_ms')} ms, overlap {b.get('overlap_pct')}%\")"
done
