#!/bin/bash
# PMC counters for one conv shape (kernel-trace only alongside --pmc, per pool rules)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
rocprofv3 -L > $R/gpurun_out/pmc_list.txt 2>&1 || true
for SH in "1024 512 1 1 14 256 fwd" "256 256 3 1 14 256 fwd"; do
  tag=$(echo $SH | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $R/gpurun_out/pmc -o sq_$tag -- python3 $R/scripts/conv_one.py $SH 10 > /dev/null 2>&1 || echo "pmc1 failed $SH"
  timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc -o tcc_$tag -- python3 $R/scripts/conv_one.py $SH 10 > /dev/null 2>&1 || echo "pmc2 failed $SH"
done
ls $R/gpurun_out/pmc
