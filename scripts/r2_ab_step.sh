set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
for g in 0 -1; do
  DPE_HGEMM_GROUP=$g timeout -k 10 200 python bench.py --model gpt2 > gpurun_out/abstep.log 2>&1 || exit 1
  echo "group=$g $(tail -1 gpurun_out/abstep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
done
