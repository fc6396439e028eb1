#!/bin/bash
# PMC counters for GEMM shapes: ours (gemm256 forced) vs torch (hipBLASLt). kernel-trace only alongside --pmc.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
mkdir -p $R/gpurun_out/pmcg
for SH in "fwd 8192 50304 768 10 2" "torch 8192 50304 768 10 0" "fwd 8192 3072 768 20 2"; do
  tag=$(echo $SH | tr ' ' '_')
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmcg -o a_$tag -- python3 $R/scripts/gemm_one.py $SH > /dev/null 2>&1 || { echo "pmc a failed $SH"; exit 1; }
  timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_LDS --kernel-trace --output-format csv -d $R/gpurun_out/pmcg -o b_$tag -- python3 $R/scripts/gemm_one.py $SH > /dev/null 2>&1 || { echo "pmc b failed $SH"; exit 1; }
done
ls $R/gpurun_out/pmcg
