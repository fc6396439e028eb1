set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
for SH in "1024 256 1 1 14 512 wgrad" "512 128 1 1 28 512 wgrad"; do
  tag=$(echo $SH | tr ' ' '_')
  timeout -k 10 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc_wg -o sq1_$tag -- python3 scripts/conv_one.py $SH 10 > /dev/null 2>&1 || exit 1
  timeout -k 10 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $R/gpurun_out/pmc_wg -o sq2_$tag -- python3 scripts/conv_one.py $SH 10 > /dev/null 2>&1 || exit 1
done
python3 scripts/pmc_summary.py gpurun_out/pmc_wg wgrad > gpurun_out/pmc_wgrad.txt
cat gpurun_out/pmc_wgrad.txt
python3 - <<'PY'
import csv, glob, collections
for f in glob.glob("gpurun_out/pmc_wg/**/*kernel_trace.csv", recursive=True):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "dpe::" in r["Kernel_Name"]:
            d[r["Kernel_Name"].split("(")[0][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in d.items(): print(f.split("/")[-1][:40], k, "median us", sorted(v)[len(v)//2])
PY
