set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for lay in fwd wgrad; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/pmc/$lay -o run -- python3 $R/scripts/hgemm_one.py $lay 8192 8192 8192 0 3 > $R/gpurun_out/pmc/$lay.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc/${lay}2 -o run -- python3 $R/scripts/hgemm_one.py $lay 8192 8192 8192 0 3 > $R/gpurun_out/pmc/${lay}2.log 2>&1 || exit 1
done
echo pmc done
