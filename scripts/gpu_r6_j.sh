#!/bin/bash
# Stall counters of the 128x128 BN-partials data-grad tile: strided parity sub-GEMMs vs the stride-1 conv.
set -o pipefail
for m in phase s1; do
  FILTER=igemm_dma bash scripts/gpu_pmc_kernels.sh scripts/pmc_phase_probe.py $m > /dev/null || exit 1
  echo "== $m"; cat gpurun_out/pmck/summary.txt
  grep -h "igemm_dma" gpurun_out/pmck/a/*kernel_trace.csv 2>/dev/null | head -0
done
