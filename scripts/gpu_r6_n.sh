#!/bin/bash
# LDS-DMA conv tile forced for every conv (DPE_CONV_TILE 0 auto / 2 256x128 / 3 256x256), ResNet-50 bench.
set -o pipefail
for r in 1 2; do
  for t in 0 2 3; do
    DPE_CONV_TILE=$t timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/tile.log 2>&1 || { tail -5 gpurun_out/tile.log; exit 1; }
    echo "tile=$t $(grep '"metric"' gpurun_out/tile.log | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["value"], l["ms_per_step"])')"
  done
done
