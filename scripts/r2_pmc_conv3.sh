# PMC counters of the 3x3 forward convs: layer1 (C=64 @56, ~490 TF) vs layer3 (C=256 @14, ~800 TF)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
: > gpurun_out/pmc_conv3.txt
for SH in "64 64 3 1 56 512 fwd" "256 256 3 1 14 512 fwd"; do
  tag=$(echo $SH | tr ' ' '_')
  timeout -k 10 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS --kernel-trace --output-format csv -d $R/gpurun_out/pmc_c3/$tag/a -o a -- python3 scripts/conv_one.py $SH 10 > /dev/null 2>&1 || exit 1
  timeout -k 10 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $R/gpurun_out/pmc_c3/$tag/b -o b -- python3 scripts/conv_one.py $SH 10 > /dev/null 2>&1 || exit 1
  timeout -k 10 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace --output-format csv -d $R/gpurun_out/pmc_c3/$tag/c -o c -- python3 scripts/conv_one.py $SH 10 > /dev/null 2>&1 || exit 1
  python3 scripts/pmc_summary.py gpurun_out/pmc_c3/$tag "$SH" >> gpurun_out/pmc_conv3.txt
done
cat gpurun_out/pmc_conv3.txt
