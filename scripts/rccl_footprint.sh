# Resource footprint of RCCL's collective kernels (threads, LDS, VGPRs, grid = channels) while the
# DDP reducer all-reduces gradient buckets at world 2 on one GPU (two ranks, distinct NCCL_HOSTID).
# Rank 0 runs under rocprofv3 --kernel-trace; the summary says how many of our persistent-kernel
# slots one RCCL channel block displaces (parallel/cu_budget.py).  Usage: bash scripts/rccl_footprint.sh [channels]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
PORT=$((29500 + RANDOM % 1000))
CH=${1:-}
common="WORLD_SIZE=2 LOCAL_RANK=0 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 OMP_NUM_THREADS=1"
args="--gpus 2 --model resnet50 --batch-size 64 --steps 4 --warmup 2 ${CH:+--comm-max-channels $CH}"
env $common RANK=1 NCCL_HOSTID=dpe-fp-1 timeout -k 10 300 python3 $R/bench.py $args > $R/gpurun_out/fp_r1.log 2>&1 &
p1=$!
env $common RANK=0 NCCL_HOSTID=dpe-fp-0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/fp_trace -o run -- python3 $R/bench.py $args > $R/gpurun_out/fp_r0.log 2>&1
rc=$?
wait $p1 || rc=$?
[ $rc -ne 0 ] && { tail -20 $R/gpurun_out/fp_r0.log $R/gpurun_out/fp_r1.log; exit $rc; }
f=$(find $R/gpurun_out/fp_trace -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'EOF'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
first = None
seen = collections.OrderedDict()
for r in rows:
    n = r["Kernel_Name"]
    if "nccl" in n.lower() or "rccl" in n.lower():
        first = first or r
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        seen.setdefault(n[:90], []).append(d)
if first:
    print({k: v for k, v in first.items() if "Timestamp" not in k and "Id" not in k})
for n, ds in seen.items():
    ds.sort()
    print(f"{n} | calls {len(ds)} | median {ds[len(ds) // 2]:.1f} us")
EOF
rm -f $f
