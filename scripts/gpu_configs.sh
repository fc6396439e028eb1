#!/bin/bash
# Every BASELINE.json config path on one GPU (bench JSON lines + a train.py run through the launcher).
set -o pipefail
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/cfg_$name.log 2>&1 || { echo "$name FAILED"; tail -20 gpurun_out/cfg_$name.log; exit 1; }; echo "$name: $(tail -1 gpurun_out/cfg_$name.log | cut -c1-330)"; }
run r50_accum8 python bench.py --grad-accum 8 --steps 3 --warmup 1
run r50_overlap python bench.py --force-comm --bucket-timing --steps 10 --warmup 3
run gpt2 python bench.py --model gpt2
run simplenet python bench.py --model simplenet --steps 50 --warmup 10
run train_simplenet python -m distributed_pytorch_example_amd.launch --nproc-per-node 1 --master-addr 127.0.0.1 train.py --epochs 2 --num-samples 10000 --checkpoint-dir /tmp/ck_s
run train_r50 python -m distributed_pytorch_example_amd.launch --nproc-per-node 1 --master-addr 127.0.0.1 train.py --model resnet50 --batch-size 128 --epochs 1 --num-samples 1024 --optimizer sgd --lr 0.1 --checkpoint-dir /tmp/ck_r
