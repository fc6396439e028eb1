#!/bin/bash
# PMC counters: 128-tile igemm vs hipBLASLt on a conv-sized dense GEMM (kernel-trace only alongside --pmc)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
mkdir -p $R/gpurun_out/pmcg2
for SH in "fwd 50176 256 2304 20 1" "torch 50176 256 2304 20 0"; do
  tag=$(echo $SH | tr ' ' '_')
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmcg2 -o a_$tag -- python3 $R/scripts/gemm_one.py $SH > /dev/null 2>&1 || { echo "pmc a failed $SH"; exit 1; }
  timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM --kernel-trace --output-format csv -d $R/gpurun_out/pmcg2 -o b_$tag -- python3 $R/scripts/gemm_one.py $SH > /dev/null 2>&1 || { echo "pmc b failed $SH"; exit 1; }
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA --kernel-trace --output-format csv -d $R/gpurun_out/pmcg2 -o c_$tag -- python3 $R/scripts/gemm_one.py $SH > /dev/null 2>&1 || { echo "pmc c failed $SH"; exit 1; }
done
ls $R/gpurun_out/pmcg2 | wc -l
