#!/bin/bash
# PMC counters (3 passes, kernel-trace only) for one conv pass shape; summary -> gpurun_out/pmc_conv.txt
# usage: SH="256 256 3 1 14 512 fwd" bash scripts/gpu_pmc_conv.sh
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
SH=${SH:-"256 256 3 1 14 512 fwd"}
tag=$(echo $SH | tr ' ' '_')
rm -rf $R/gpurun_out/pmc; mkdir -p $R/gpurun_out/pmc
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $R/gpurun_out/pmc -o p$i -- python3 $R/scripts/conv_one.py $SH 10 > $R/gpurun_out/pmc/log$i.txt 2>&1 || { echo "pmc pass $i failed"; tail -5 $R/gpurun_out/pmc/log$i.txt; exit 1; }
done
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc "$SH" | tee $R/gpurun_out/pmc_conv_$tag.txt
