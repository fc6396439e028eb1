set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for lay in fwd wgrad dgrad; do
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum --output-format csv -d $R/gpurun_out/pmc/${lay}3 -o run -- python3 $R/scripts/hgemm_one.py $lay 8192 8192 8192 0 3 > $R/gpurun_out/pmc/${lay}3.log 2>&1 || exit 1
done
echo pmc done
