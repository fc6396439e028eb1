# TA / TD / TCP pipeline counters of the layer-1 3x3 forward conv (LDS-DMA kernel, 256x64 tile)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
SH="64 64 3 1 56 512 fwd"
timeout -k 10 60 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_SPI_STALL_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_ta/a -o a -- python3 scripts/conv_one.py $SH 10 > gpurun_out/pmc_ta_a.log 2>&1 || { tail gpurun_out/pmc_ta_a.log; exit 1; }
timeout -k 10 60 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_ta/b -o b -- python3 scripts/conv_one.py $SH 10 > gpurun_out/pmc_ta_b.log 2>&1 || { tail gpurun_out/pmc_ta_b.log; exit 1; }
timeout -k 10 60 rocprofv3 --pmc TCC_BUSY_sum TCC_TAG_STALL_sum TCC_REQ_sum GRBM_GUI_ACTIVE SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM --kernel-trace --output-format csv -d $R/gpurun_out/pmc_ta/c -o c -- python3 scripts/conv_one.py $SH 10 > gpurun_out/pmc_ta_c.log 2>&1 || { tail gpurun_out/pmc_ta_c.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_ta "$SH" > gpurun_out/pmc_ta.txt
cat gpurun_out/pmc_ta.txt
