set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
timeout -k 10 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc_attn -o sq1 -- python3 scripts/bench_attn.py --reps 3 > gpurun_out/pmc1.log 2>&1 || exit 1
timeout -k 10 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $R/gpurun_out/pmc_attn -o sq2 -- python3 scripts/bench_attn.py --reps 3 > gpurun_out/pmc2.log 2>&1 || exit 1
python3 scripts/pmc_summary.py gpurun_out/pmc_attn attn > gpurun_out/pmc_attn.txt
